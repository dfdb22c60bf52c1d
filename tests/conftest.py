import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
for p in (REPO / "raytracer-cuda_amd", REPO / "oracle", REPO):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def scenes():
    from crt_amd import assets
    return {k: assets.scene_files(k) for k in ("cornell", "cornell_bunny")}


@pytest.fixture(scope="session")
def oracle_scenes(scenes):
    import objload
    import pyoracle
    return {k: pyoracle.OracleScene(objload.load_scene(v)) for k, v in scenes.items()}


@pytest.fixture(scope="session")
def device_scenes(scenes):
    import crt_amd
    out = {}
    for k, v in scenes.items():
        hs = crt_amd.HostScene(v)
        out[k] = (hs, hs.upload(0))
    return out

"""Every `File:line` citation of the reference in this repository's product, oracle and design files points inside
the cited reference file (CPU).

The line counts come from tests/golden/reference_file_lines.json (make_reference_lines.py over
/root/reference/CudaRayTracer/src); when the reference is present the table is checked against it too.  A citation is
`Name.ext:A` or `Name.ext:A-B`, optionally continued by `, :C-D` for the same file.
"""
import json
import re
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
TABLE = json.loads((REPO / "tests" / "golden" / "reference_file_lines.json").read_text())
SCANNED = (["DESIGN.md", "INTEGRATION.md", "bench.py", "__graft_entry__.py"]
           + [str(p.relative_to(REPO)) for d in ("oracle", "include", "raytracer-cuda_amd/csrc", "raytracer-cuda_amd/host",
                                                 "raytracer-cuda_amd/crt_amd")
              for p in sorted((REPO / d).rglob("*")) if p.suffix in (".c", ".h", ".hip", ".cpp", ".py", ".md")])
CITE = re.compile(r"\b([A-Za-z_]+\.(?:cuh|h|cu))((?::\d+(?:-\d+)?)(?:,\s*:\d+(?:-\d+)?)*)")


def citations(text):
    for m in CITE.finditer(text):
        name = m.group(1)
        if name not in TABLE:
            continue
        for a, b in re.findall(r":(\d+)(?:-(\d+))?", m.group(2)):
            yield name, int(a), int(b) if b else int(a), m.group(0)


def test_table_matches_reference():
    src = Path("/root/reference/CudaRayTracer/src")
    if not src.exists():
        pytest.skip("reference not present (GPU box)")
    for name, e in TABLE.items():
        data = (Path("/root/reference") / e["path"]).read_bytes()
        assert len(data.split(b"\n")) - (1 if data.endswith(b"\n") else 0) == e["lines"], name


def test_citations_fall_inside_the_cited_files():
    bad, n = [], 0
    for rel in SCANNED:
        text = (REPO / rel).read_text(errors="replace")
        for name, a, b, raw in citations(text):
            n += 1
            if not (1 <= a <= b <= TABLE[name]["lines"]):
                bad.append(f"{rel}: {raw} ({name} has {TABLE[name]['lines']} lines)")
    assert n > 100, n      # the scan really sees the citations
    assert not bad, "\n".join(bad)

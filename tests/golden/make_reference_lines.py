"""Writes tests/golden/reference_file_lines.json: the line count of every source file of the reference
(/root/reference/CudaRayTracer/src), keyed by basename — the data test_citations.py checks every `File:line`
citation in this repository against (the reference itself does not travel to the GPU box)."""
import json
from pathlib import Path

SRC = Path("/root/reference/CudaRayTracer/src")
OUT = Path(__file__).resolve().parent / "reference_file_lines.json"

if __name__ == "__main__":
    table = {}
    for p in sorted(SRC.rglob("*")):
        if p.suffix in (".cuh", ".h", ".cu", ".cpp") and p.is_file():
            n = len(p.read_bytes().split(b"\n"))
            if p.read_bytes().endswith(b"\n"):
                n -= 1
            assert p.name not in table, f"duplicate basename {p.name}"
            table[p.name] = {"path": str(p.relative_to(SRC.parents[1])), "lines": n}
    OUT.write_text(json.dumps(table, indent=1, sort_keys=True) + "\n")
    print(f"{len(table)} files -> {OUT}")

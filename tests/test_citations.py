"""Every reference citation in the product, oracle, tests and docs resolves to real lines.

Citations are the audit trail of the restatement (`AF:318-344`, `MNcs:151-152`, `MipHelpers.cs:403`):
a line past the end of the cited file means the trail is wrong even when the math is right.  The
check reads the reference tree as text (line counts only); it is skipped where the tree is absent
(the GPU box).
"""
from __future__ import annotations

import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/ScratchNerf"
# SURVEY.md's abbreviations
ABBREV = {
    "AF": "AcceleratedNeRFUtils/accelerated_functions.cu",
    "MLPcpp": "AcceleratedNeRFUtils/AcceleratedMLP.cpp",
    "MNcpp": "AcceleratedNeRFUtils/AcceleratedMipNeRF.cpp",
    "MH": "ScratchNerf/MipHelpers.cs",
    "MLPcs": "ScratchNerf/MLP.cs",
    "MNcs": "ScratchNerf/MipNerfModel.cs",
}
SCAN_DIRS = ["nerf-or-nothing_amd/csrc", "nerf-or-nothing_amd/nof", "nerf-or-nothing_amd/app", "oracle", "include",
             "tests"]
SCAN_FILES = ["DESIGN.md", "INTEGRATION.md", "README.md", "bench.py", "__graft_entry__.py"]
EXTS = (".hip", ".h", ".cpp", ".py", ".md", ".c")
CITE = re.compile(r"\b([A-Za-z][A-Za-z0-9_.]*?(?:\.cs|\.cpp|\.cu|\.h)|AF|MLPcpp|MNcpp|MH|MLPcs|MNcs):"
                  r"(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)")


def _ref_lengths():
    n = {}
    for d, _, fs in os.walk(REF):
        for f in fs:
            p = os.path.join(d, f)
            with open(p, "rb") as fh:
                n.setdefault(f, []).append(fh.read().count(b"\n") + 1)
    return n


def _sources():
    for d in SCAN_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            for f in fs:
                if f.endswith(EXTS) and f != os.path.basename(__file__):
                    yield os.path.join(dp, f)
    for f in SCAN_FILES:
        yield os.path.join(ROOT, f)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_reference_citations_resolve():
    lengths = _ref_lengths()
    bad, checked = [], 0
    for path in _sources():
        if not os.path.exists(path):
            continue
        text = open(path, encoding="utf-8", errors="replace").read()
        for m in CITE.finditer(text):
            name, spans = m.group(1), m.group(2)
            fname = os.path.basename(ABBREV[name]) if name in ABBREV else os.path.basename(name)
            if fname not in lengths:
                continue  # not a reference file (e.g. one of this repo's own sources)
            top = max(lengths[fname])
            for span in spans.split(","):
                lo, _, hi = span.partition("-")
                lo, hi = int(lo), int(hi or lo)
                checked += 1
                if not (1 <= lo <= hi <= top):
                    line = text.count("\n", 0, m.start()) + 1
                    bad.append(f"{os.path.relpath(path, ROOT)}:{line}: {name}:{span} ({fname} has {top} lines)")
    assert checked > 200, f"only {checked} citations found: the pattern no longer matches the sources"
    assert not bad, "citations past the end of the cited file:\n" + "\n".join(bad)

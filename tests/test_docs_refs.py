"""The documents cite files for their numbers (profiles, scripts, tests): every
path they name in backticks must exist in the tree, so that a figure in
DESIGN.md or INTEGRATION.md can be traced to the file it came from.  CPU
only; forms with an ellipsis, a placeholder or a glob are skipped."""
from __future__ import annotations

import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = "klt-feature-tracker-acceleration-gpus_amd"
DOCS = ("DESIGN.md", "INTEGRATION.md", "tools/exp/INDEX.md")
# bare file names resolve against these directories
SEARCH = ("", "profiles/", "archive/profiles/", "tools/", "tools/exp/", "tools/exp/patches/", "archive/tools_exp/",
          "tests/", "tests/golden/", "oracle/", f"{PKG}/", f"{PKG}/csrc/")
# names of files outside this tree (the reference's own tooling)
EXTERNAL = {"gprof2dot.py"}


def _skip(p: str) -> bool:
    return any(ch in p for ch in "…<>{}*$")


def test_cited_paths_exist():
    missing = []
    for doc in DOCS:
        text = (ROOT / doc).read_text()
        for m in re.finditer(r"`((?:profiles|tools|tests|oracle|include|archive|" + re.escape(PKG) + r")/[^`\s]+)`",
                             text):
            p = m.group(1).rstrip(".,;:)").split("::")[0]
            if not _skip(p) and not (ROOT / p).exists():
                missing.append((doc, p))
        for m in re.finditer(r"`([\w.-]+\.(?:txt|json|csv|patch|sh|py))`", text):
            name = m.group(1)
            if name in EXTERNAL or _skip(name):
                continue
            if not any((ROOT / (d + name)).exists() for d in SEARCH):
                missing.append((doc, name))
    assert not missing, missing

"""Every profiles/ path DESIGN.md, INTEGRATION.md and README.md cite exists in the tree or is cited as
<commit>:<path> at a commit that holds it (tools/check_citations.py; ADVICE r05: a pruning commit left
32 citations dangling)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_profile_citations_resolve():
    if not shutil.which("git") or not os.path.isdir(os.path.join(ROOT, ".git")):
        pytest.skip("needs the git history (the GPU box's snapshot has none)")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_citations
    assert check_citations.check() == []

"""The evidence tree stays auditable (VERDICT r5 Next #7): every committed file under
profiles/ and tools/sessions/ is cited by a tracked document or by the code whose constants
it backs, so nothing under them is an orphaned A/B leftover."""
from __future__ import annotations

import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tracked() -> list[str]:
    p = subprocess.run(["git", "ls-files"], cwd=REPO, capture_output=True, text=True)
    if p.returncode != 0:
        pytest.skip("not a git checkout")
    return [f for f in p.stdout.split() if os.path.exists(os.path.join(REPO, f))]


def _names(f: str) -> list[str]:
    """How a document may name a file: its repo path, the path below profiles/ or below its
    round directory, or its file name."""
    parts = f.split("/")
    return [c for c in {f, parts[-1], "/".join(parts[1:]), "/".join(parts[2:])} if len(c) > 3]


def test_every_evidence_file_is_cited():
    files = _tracked()
    evidence = [f for f in files
                if (f.startswith("profiles/") or f.startswith("tools/sessions/"))
                and not f.endswith("README.md")]
    citing = [f for f in files if f.endswith(".md") or
              f.rsplit(".", 1)[-1] in ("py", "cpp", "hpp", "hip", "inc", "sh")]
    text = {}
    for f in citing:
        with open(os.path.join(REPO, f), errors="replace") as fh:
            text[f] = fh.read()
    orphans = []
    for f in evidence:
        # a document does not count as citing itself
        if not any(n in t for n in _names(f) for g, t in text.items() if g != f):
            orphans.append(f)
    assert not orphans, f"uncited evidence files: {orphans}"


def test_profile_index_names_only_existing_documents():
    """profiles/README.md indexes documents that exist (no stale rows after a prune)."""
    import re

    with open(os.path.join(REPO, "profiles", "README.md")) as f:
        readme = f.read()
    for ref in re.findall(r"`(r\d/[^`]+\.(?:md|json))`", readme):
        assert os.path.exists(os.path.join(REPO, "profiles", ref)), ref

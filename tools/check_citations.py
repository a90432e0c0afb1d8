#!/usr/bin/env python3
"""Check (or, with --fix, repair) the profiles/ citations of DESIGN.md, INTEGRATION.md and README.md:
every cited path must exist in the tree, or be cited as <commit>:<path> (git's rev:path syntax) at a
commit that holds it. --fix rewrites a dangling path to <commit>:<path>, where <commit> is the parent
of the commit that deleted it."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ("DESIGN.md", "INTEGRATION.md", "README.md")
PAT = re.compile(r"(?:(?<![\w/])([0-9a-f]{7,40}):)?(profiles/[A-Za-z0-9_./\-]*[A-Za-z0-9_/\-])")


def git(*a):
    return subprocess.run(["git", "-C", ROOT, *a], capture_output=True, text=True)


def in_commit(rev, path):
    return git("cat-file", "-e", f"{rev}:{path.rstrip('/')}").returncode == 0


def deleted_at(path):
    r = git("rev-list", "-1", "HEAD", "--", path.rstrip("/"))
    c = r.stdout.strip()
    if not c:
        return None
    parent = git("rev-parse", "--short", c + "^").stdout.strip()
    return parent if parent and in_commit(parent, path) else None


def check(fix=False):
    bad = []
    for doc in DOCS:
        p = os.path.join(ROOT, doc)
        s = open(p).read()
        out, pos = [], 0
        for m in PAT.finditer(s):
            rev, path = m.group(1), m.group(2)
            nxt = s[m.end(2):m.end(2) + 1]
            if path.rstrip("/") in ("profiles", "profiles/r0") or nxt in ("*", "{"):   # the directory / a pattern
                continue
            if rev:
                if not in_commit(rev, path):
                    bad.append(f"{doc}: {rev}:{path} not in that commit")
                continue
            if os.path.exists(os.path.join(ROOT, path)):
                continue
            c = deleted_at(path) if fix else None
            if c:
                out.append(s[pos:m.start(2)] + f"{c}:{path}")
                pos = m.end(2)
            else:
                bad.append(f"{doc}: {path} missing")
        if fix:
            out.append(s[pos:])
            open(p, "w").write("".join(out))
    return bad


if __name__ == "__main__":
    bad = check(fix="--fix" in sys.argv)
    print("\n".join(bad) if bad else "ok")
    sys.exit(1 if bad else 0)

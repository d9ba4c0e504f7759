"""DESIGN.md is the current-state design document: every profile it cites
exists under profiles/ (cited as `profiles/NAME` or, after one such citation
in the same sentence, by a bare `rNN_...` name), and it stays short enough to
read (the round-by-round record is HISTORY.md)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _design():
    with open(os.path.join(ROOT, "DESIGN.md")) as f:
        return f.read()


def test_design_cites_existing_profiles():
    txt = _design()
    names = set(re.findall(r"profiles/([A-Za-z0-9_.{},\-*]+)", txt))
    names |= set(re.findall(r"`(r0\d_[A-Za-z0-9_.\-]+\.(?:log|json|jsonl|csv|txt))`", txt))
    missing = []
    for n in sorted(names):
        n = n.rstrip(".,")
        if n.endswith("/") or not n:
            continue
        if not os.path.exists(os.path.join(ROOT, "profiles", n)):
            missing.append(n)
    assert not missing, missing


def test_design_is_current_state_sized():
    assert len(_design().splitlines()) <= 700

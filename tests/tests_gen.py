"""Input records of the golden edge cases (regenerated deterministically by
the same code that made the fixtures, tests/golden/make_golden.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden  # noqa: E402

_CASES = None


def edge_records(name: str):
    global _CASES
    if _CASES is None:
        _CASES = make_golden.edge_cases()
    return _CASES[name][0]

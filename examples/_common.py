"""Shared helpers for the examples: synthetic stand-ins for the reference examples' datasets (this sandbox has
no network access, so the iris / adult / MovieLens / avazu files are generated with the same schemas)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def args(default_rows):
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default=None, help="cpu or cuda:0 (default: cuda when available)")
    ap.add_argument("--rows", type=int, default=default_rows)
    ap.add_argument("--workdir", default=os.environ.get("TMPDIR", "/tmp"))
    return ap.parse_args()

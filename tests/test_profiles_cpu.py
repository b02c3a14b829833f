"""Committed measurement records stay machine-readable: every
profiles/*.json parses as JSON (one started with Gloo stderr)."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "profiles", "*.json")))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_profile_json_parses(path):
    with open(path) as f:
        json.load(f)

"""The GPU suite's time budget: the driver runs
`pytest -m gpu` on one MI355X within a 900 s step, and the suite is kept
under ~600 s.  Every GPU test function states its measured duration on the
driver's box in its docstring — "(~N s)" for all its parameter cases
together — so a new case shows its cost where it is added, and this check
adds them up.  Cases beyond parity coverage (repeats, soaks, long late-rank
waits) carry @pytest.mark.slow and are deselected by default (conftest.py);
their notes do not count."""
import ast
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NOTE = re.compile(r"\(~\s*(\d+(?:\.\d+)?)\s*(s|min)\b")
BUDGET_S = 600


def _marks(dec):
    """Names of pytest.mark.<name> decorators (called or not)."""
    out = set()
    for d in dec:
        node = d.func if isinstance(d, ast.Call) else d
        if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Attribute) and node.value.attr == "mark":
            out.add(node.attr)
    return out


def _gpu_tests():
    for path in sorted(glob.glob(os.path.join(ROOT, "tests", "test_*.py"))):
        tree = ast.parse(open(path).read(), path)
        module_gpu = any(isinstance(n, ast.Assign) and any(getattr(t, "id", "") == "pytestmark" for t in n.targets)
                         and "gpu" in ast.unparse(n.value) for n in tree.body)
        for fn in tree.body:
            if isinstance(fn, ast.FunctionDef) and fn.name.startswith("test_"):
                marks = _marks(fn.decorator_list)
                if module_gpu or "gpu" in marks:
                    yield os.path.basename(path), fn, marks


def test_every_gpu_test_states_its_duration():
    missing = [f"{mod}::{fn.name}" for mod, fn, _ in _gpu_tests() if not NOTE.search(ast.get_docstring(fn) or "")]
    assert not missing, f"GPU tests without a '(~N s)' duration note in their docstring: {missing}"


def test_default_gpu_selection_fits_the_budget():
    total = 0.0
    for _, fn, marks in _gpu_tests():
        if "slow" in marks:
            continue
        m = NOTE.search(ast.get_docstring(fn) or "")
        if m:
            total += float(m.group(1)) * (60 if m.group(2) == "min" else 1)
    assert total <= BUDGET_S, f"default -m gpu selection adds up to ~{total:.0f} s (budget {BUDGET_S} s)"

"""The CI lint job (tools/lint.py) stays clean: syntax, unused imports,
whitespace, line length, and no CUDA spellings in the gfx950 sources."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lint_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lint.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:]

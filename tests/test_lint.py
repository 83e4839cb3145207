"""CI lint step (reference: flake8 in tox.ini:4-5 / peteris.yaml): the Python tree is clean
under tools/lint.py (flake8's rule subset, see tox.ini)."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import lint  # noqa: E402


def test_tree_is_lint_clean(capsys):
    assert lint.main([]) == 0, capsys.readouterr().out


def test_lint_detects_problems(tmp_path):
    p = tmp_path / "bad.py"
    p.write_text("import os\nimport sys\ntry:\n    pass\nexcept:  \n    pass\nx = sys.argv" + " " * 130 + "\n")
    codes = {line.split()[1] for line in lint.lint_file(str(p))}
    assert codes == {"F401", "E722", "W291", "E501"}

"""The repository passes its own lint (scripts/lint.py, run by CI and pre-commit)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scripts"))
import lint  # noqa: E402


def test_repository_is_lint_clean():
    problems = lint.lint()
    assert not problems, "\n".join(f"{f}:{ln}: {m}" for f, ln, m in problems[:30])


def test_lint_flags_dual_platform_code(tmp_path):
    bad = tmp_path / "k.hip"
    bad.write_text("#ifdef __HIP_PLATFORM_AMD__\nint x;\n#endif\n")
    probs = lint.lint([str(bad)])
    assert any("dual-platform" in m for _, _, m in probs)
    py = tmp_path / "m.py"
    py.write_text("import os\nimport sys\nprint(sys.argv)\n")
    assert [m for _, _, m in lint.lint([str(py)])] == ["unused import 'os'"]

"""The README's "Python API in brief" names only what the package exports: every `ops.X` / `P.X` attribute and every
method called on the documented objects exists (a docs-drift check; no GPU needed)."""
import re
from pathlib import Path

import pytest

from parallel_c_programs_amd import ops
from parallel_c_programs_amd import parallel as P

README = Path(__file__).resolve().parents[1] / "README.md"


def _api_block() -> str:
    text = README.read_text()
    start = text.index("## Python API in brief")
    block = text[start:]
    return block[block.index("```python") + len("```python"):block.index("```", block.index("```python") + 9)]


def test_readme_api_block_names_exist():
    code = _api_block()
    for mod, name in re.findall(r"\b(ops|P)\.([A-Za-z_][A-Za-z0-9_]*)", code):
        assert hasattr(ops if mod == "ops" else P, name), f"README names {mod}.{name}, which does not exist"


@pytest.mark.parametrize("cls,methods", [
    ("StencilSlab", ["run", "step", "interior", "gather"]),
    ("DistributedSpMV", ["powerlaw", "iterate", "to_padded", "from_padded", "step"]),
])
def test_readme_documented_methods_exist(cls, methods):
    c = getattr(P, cls)
    for m in methods:
        assert hasattr(c, m), f"{cls}.{m}"


def test_readme_prose_names_exist():
    text = README.read_text()
    prose = text[text.index("## Python API in brief"):text.index("## Tests")]
    for name in re.findall(r"`([A-Za-z_][A-Za-z0-9_]*)`", prose.split("```", 2)[-1]):
        if name in ("ops", "parallel"):  # the module names themselves
            continue
        assert hasattr(P, name) or hasattr(ops, name), f"README prose names `{name}`"

"""Fixtures, oracles, stdout formats."""
from . import fixtures, oracle, output  # noqa: F401

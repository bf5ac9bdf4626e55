"""Integrand workloads (the reference's 'models'): see integrands.py."""
from .integrands import IntegrandSpec, get, pi4, poly, sin, table, train  # noqa: F401

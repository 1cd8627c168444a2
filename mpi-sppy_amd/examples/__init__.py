"""Pyomo-free scenario creators restating the reference examples (``examples/*``)."""

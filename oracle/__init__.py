"""ORACLE — test infrastructure only (see loader.py)."""

"""ORACLE — test infrastructure only (see ed25519_oracle.c). Importable by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product package."""

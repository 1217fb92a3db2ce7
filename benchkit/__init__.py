"""Measurement plumbing of bench.py (the contract entry point stays bench.py at the repository root)."""

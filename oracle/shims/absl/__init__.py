"""Stand-in for absl (logging only) — oracle/make_golden.py import shim, no arithmetic."""

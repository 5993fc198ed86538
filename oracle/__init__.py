"""Parity oracle (test infrastructure only; never imported by preganplus_amd)."""

"""Test-only empty stand-in for h5py (only the reference\x27s h5py I/O paths use it)."""

"""Run pytest with torch.empty() filled with NaN (deterministic mode), so a
kernel reading memory it never wrote fails every time instead of sometimes.
usage: python tools/nan_probe.py <pytest args>"""
import sys, torch
torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
import pytest
sys.exit(pytest.main(sys.argv[1:]))

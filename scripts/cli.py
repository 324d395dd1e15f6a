"""CLI base class for task scripts (reference scripts/cli.py) — see perceiver_io_amd/cli."""
import _bootstrap  # noqa: F401

from perceiver_io_amd.cli import CLI, freeze  # noqa: F401

try:  # `python scripts/x.py` puts scripts/ on sys.path (reference scripts/__init__.py:1)
    from cli import CLI  # noqa: F401
except ImportError:  # imported as a package from the repository root
    from perceiver_io_amd.cli import CLI  # noqa: F401

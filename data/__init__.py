"""``data`` compatibility package (reference ``data/__init__.py``); importing it registers the
data modules for ``--data=<ClassName>``."""
from perceiver_io_amd.data import IMDBDataModule, MNISTDataModule, SyntheticImageDataModule  # noqa: F401

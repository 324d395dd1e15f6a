from perceiver_io_amd.data.mnist import MNISTDataModule  # noqa: F401

"""Data-module registry (``--data=<ClassName>``; reference ``DATAMODULE_REGISTRY``,
``data/imdb.py:71``, ``data/mnist.py:8``)."""
DATAMODULE_REGISTRY = {}


def register_datamodule(cls):
    DATAMODULE_REGISTRY[cls.__name__] = cls
    return cls

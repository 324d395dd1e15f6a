from perceiver_io_amd.data.imdb import Collator, IMDBDataModule, IMDBDataset, load_split  # noqa: F401

"""Data modules: IMDB (text), MNIST (images), synthetic ImageNet-shape images, LArTPC-shape events."""
from .imdb import Collator, IMDBDataModule, IMDBDataset, load_split
from .mnist import MNISTDataModule, SyntheticImageDataModule
from .registry import DATAMODULE_REGISTRY, register_datamodule
from .synthetic import SyntheticImages, SyntheticLArTPC, SyntheticText, lartpc_event

__all__ = ["Collator", "IMDBDataModule", "IMDBDataset", "load_split", "MNISTDataModule", "SyntheticImageDataModule",
           "DATAMODULE_REGISTRY", "register_datamodule", "SyntheticImages", "SyntheticLArTPC", "SyntheticText",
           "lartpc_event"]

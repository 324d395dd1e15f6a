"""Training stack: LightningModule-compatible base, Trainer, step engine (hipGraph), callbacks,
loggers, Lightning-layout checkpoints."""
from .callbacks import Callback, EarlyStopping, LearningRateMonitor, ModelCheckpoint
from .checkpoint import load_checkpoint, make_checkpoint, save_checkpoint
from .engine import StepEngine
from .loggers import CSVLogger, TensorBoardLogger
from .module import LitModuleBase, instantiate_class
from .trainer import Trainer

__all__ = ["Callback", "EarlyStopping", "LearningRateMonitor", "ModelCheckpoint", "load_checkpoint", "make_checkpoint",
           "save_checkpoint", "StepEngine", "CSVLogger", "TensorBoardLogger", "LitModuleBase", "instantiate_class",
           "Trainer"]

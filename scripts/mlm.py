"""Masked-language-model pretraining (IMDB) — `python scripts/mlm.py {fit,validate,test} --model.* --data=... --trainer.* ...`
(reference scripts/mlm.py; links/defaults in perceiver_io_amd/cli/tasks.py)."""
import _bootstrap  # noqa: F401

from perceiver_io_amd.cli.tasks import main

if __name__ == "__main__":
    main("mlm")

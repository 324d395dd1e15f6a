"""Sentiment classification (IMDB), optionally from an MLM encoder — `python scripts/seq_clf.py {fit,validate,test} --model.* --data=... --trainer.* ...`
(reference scripts/seq_clf.py; links/defaults in perceiver_io_amd/cli/tasks.py)."""
import _bootstrap  # noqa: F401

from perceiver_io_amd.cli.tasks import main

if __name__ == "__main__":
    main("seq_clf")

"""Image classification (MNIST / synthetic images) — `python scripts/img_clf.py {fit,validate,test} --model.* --data=... --trainer.* ...`
(reference scripts/img_clf.py; links/defaults in perceiver_io_amd/cli/tasks.py)."""
import _bootstrap  # noqa: F401

from perceiver_io_amd.cli.tasks import main

if __name__ == "__main__":
    main("img_clf")

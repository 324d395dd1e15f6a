"""Put the repository root on sys.path so ``python scripts/<task>.py`` works from anywhere
(the reference required ``export PYTHONPATH=.``)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

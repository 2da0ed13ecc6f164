"""Drop-in for the reference's ``packages/constants.py`` (driver plumbing, not the hot path):
``SCRATCH_DIR = $SCRATCH_DIR/dp_tokenization`` (created), read from the environment or a
``.env`` file when python-dotenv is installed.  Like the reference (constants.py:5-6) an unset
``SCRATCH_DIR`` raises TypeError from ``os.path.join``."""
import os

try:
    from dotenv import load_dotenv
    load_dotenv()
except ImportError:  # python-dotenv is optional here
    pass

SCRATCH_DIR = os.path.join(os.getenv("SCRATCH_DIR"), "dp_tokenization")
os.makedirs(f"{SCRATCH_DIR}", exist_ok=True)

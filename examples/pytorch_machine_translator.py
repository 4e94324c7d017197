"""sparkmi counterpart of the reference's pytorch_machine_translator.py: runs sparkmi.recipes.translator
with defaults "--world 1" (any recipe flag overrides them, e.g. --world 8 --epochs 1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sparkmi.recipes import translator  # noqa: E402

if __name__ == "__main__":
    translator.main("--world 1".split() + sys.argv[1:])

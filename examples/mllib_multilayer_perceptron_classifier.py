"""sparkmi counterpart of the reference's mllib_multilayer_perceptron_classifier.py: runs sparkmi.recipes.mllib_mlp
with defaults "" (any recipe flag overrides them, e.g. --world 8 --epochs 1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sparkmi.recipes import mllib_mlp  # noqa: E402

if __name__ == "__main__":
    mllib_mlp.main("".split() + sys.argv[1:])

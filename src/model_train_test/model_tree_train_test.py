"""Tree-model training run (reference: src/model_train_test/model_tree_train_test.py)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from cobalt_smart_lender_ai_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["train"] + sys.argv[1:]))

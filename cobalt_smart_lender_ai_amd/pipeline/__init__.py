"""Batch pipelines: data-lake preprocessing stages and the tree-model training run."""

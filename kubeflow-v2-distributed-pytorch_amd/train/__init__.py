"""Trainer: ``python -m mipipe.train.task`` (flag-compatible with the reference task.py)."""

"""Torch client algorithms with the reference's module paths and ``train`` sequence."""

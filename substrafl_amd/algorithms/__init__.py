"""Client-side bucket operations (substrafl/algorithms/pytorch/weight_manager.py mirror)."""

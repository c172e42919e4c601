"""Index generators, dense oracles and timing helpers."""

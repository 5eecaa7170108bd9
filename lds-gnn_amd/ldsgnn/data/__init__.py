"""Data preparation for the LDS hot path (SURVEY §8(f)2 "next"): synthetic
datasets of the BASELINE configs' shapes and the kNN θ initialisation."""

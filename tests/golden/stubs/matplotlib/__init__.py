"""Stand-in: predict.py imports matplotlib but the feature path never plots."""

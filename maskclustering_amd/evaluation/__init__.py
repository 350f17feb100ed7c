"""Drop-in for the device part of the reference's ``evaluation/evaluate.py``."""

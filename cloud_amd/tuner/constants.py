"""Tuner constants (reference ``TFC/tuner/constants.py:20-30``)."""
SUGGESTION_COUNT_PER_REQUEST = 1
NUM_TRIES_FOR_STUDIES = 3
MAX_TRIALS_PER_STUDY = 1000

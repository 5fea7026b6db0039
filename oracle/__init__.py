"""ORACLE — test infrastructure only (see ref_model.py header). Never imported by the shipped package."""
from .ref_model import *  # noqa: F401,F403

"""Runnable examples (``python -m myfyp_amd experiment list``)."""

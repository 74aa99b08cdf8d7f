"""In-process transport."""

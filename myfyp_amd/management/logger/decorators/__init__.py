"""Logger decorators."""

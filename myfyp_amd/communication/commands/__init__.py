"""Command pattern: every message type is a named handler."""

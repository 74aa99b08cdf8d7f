"""Weights-carrying commands (never relayed)."""

"""Utilities: topologies, seeding, sync helpers."""

"""In-memory client (parity: ``memory/memory_client.py:32-174``): a send calls the receiving
protocol's handler directly, on the sender's thread, like the reference (``memory_client.py:139``)."""

from myfyp_amd.communication.protocols.client import StubClient


class InMemoryClient(StubClient):
    """Generic stub client over in-process protocol objects."""

"""Protocol exceptions (parity: ``protocols/exceptions.py:21-36``)."""


class ProtocolNotStartedError(Exception):
    """The protocol was used before ``start()``."""


class NeighborNotConnectedError(Exception):
    """Send to a peer that is not a (direct) neighbour."""


class CommunicationError(Exception):
    """The remote side reported an error."""

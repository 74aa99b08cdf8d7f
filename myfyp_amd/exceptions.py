"""Framework exceptions (parity: ``p2pfl/exceptions.py:21-36``)."""


class NodeRunningException(Exception):
    """Raised when the node is (or is not) running and the opposite was expected."""


class LearnerRunningException(Exception):
    """Raised when learner/model/data are changed while learning is running."""


class ZeroRoundsException(Exception):
    """Raised when learning is started with fewer than one round."""

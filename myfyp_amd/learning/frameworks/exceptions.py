"""Learning exceptions (parity: ``frameworks/exceptions.py:22-31``)."""


class DecodingParamsError(Exception):
    """A serialized model could not be decoded."""


class ModelNotMatchingError(Exception):
    """Parameters do not match the model's architecture."""

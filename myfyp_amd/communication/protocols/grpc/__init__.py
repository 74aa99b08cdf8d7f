"""gRPC transport."""

"""Control-plane (small, TTL-relayed) message commands."""

"""Reference-semantics (message gossip) stages."""

"""Stage workflow (parity: ``p2pfl/stages``): Start → Vote → (Train | WaitAgg) → Gossip → RoundFinished."""

"""Learning layer: models, learners, aggregators, datasets."""

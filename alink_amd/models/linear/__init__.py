"""Linear models: objectives, distributed optimizers, training drivers, model format and mappers."""

"""Feature engineering: scalers, imputers, encoders, discretizers, hashing, PCA, selectors."""

"""alink_amd — an MI355X-native classical-ML pipeline platform with Alink's capabilities."""
__version__ = "0.1.0"

"""Tree models: GBDT, random forests and decision trees (histogram-based, level-wise, device resident)."""
from .data import BinnedData, build_bins, categorical_cols  # noqa: F401
from .engine import SplitConfig, TreeBuilder  # noqa: F401
from .model import (GbdtModelMapper, LabelCounter, Node, RandomForestModelMapper, TreeModel,  # noqa: F401
                    TreeModelDataConverter, TreeModelMapper, feature_importance)
from .train import train_forest, train_gbdt  # noqa: F401

"""Stream operators (micro-batch engine)."""
from .base import *  # noqa: F401,F403
from .utils import *  # noqa: F401,F403
from .predict import *  # noqa: F401,F403

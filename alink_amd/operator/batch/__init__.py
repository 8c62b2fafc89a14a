"""Batch operators."""
from .source import *  # noqa: F401,F403
from .sink import *  # noqa: F401,F403
from .utils import *  # noqa: F401,F403
from .dataproc import *  # noqa: F401,F403
from .clustering import *  # noqa: F401,F403
from .sql import *  # noqa: F401,F403
from .linear import *  # noqa: F401,F403
from .evaluation import *  # noqa: F401,F403
from .feature import *  # noqa: F401,F403
from .tree import *  # noqa: F401,F403
from .recommendation import *  # noqa: F401,F403
from .nlp import *  # noqa: F401,F403
from .classification_extra import *  # noqa: F401,F403
from .format import *  # noqa: F401,F403
from .regression_extra import *  # noqa: F401,F403
from .mining import *  # noqa: F401,F403
from .db import *  # noqa: F401,F403

"""Stream operators (micro-batch engine)."""
from .base import *  # noqa: F401,F403
from .utils import *  # noqa: F401,F403
from .predict import *  # noqa: F401,F403
from .source import *  # noqa: F401,F403
from .sink import *  # noqa: F401,F403
from .sql import *  # noqa: F401,F403
from .dataproc import *  # noqa: F401,F403
from .evaluation import *  # noqa: F401,F403
from .onlinelearning import *  # noqa: F401,F403
from .format import *  # noqa: F401,F403
from .db import *  # noqa: F401,F403

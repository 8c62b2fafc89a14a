from .converter import *  # noqa: F401,F403

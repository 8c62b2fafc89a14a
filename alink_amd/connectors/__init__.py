"""Connectors: Kafka (stream source / sink, universal + 0.10 + 0.11 flavours) and Hive (batch source / sink,
stream source).  See ``kafka.py`` / ``hive.py``."""
from .kafka import *  # noqa: F401,F403
from .hive import *  # noqa: F401,F403

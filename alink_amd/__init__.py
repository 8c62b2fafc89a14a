"""alink_amd — an MI355X-native classical-ML pipeline platform with Alink's capabilities.

``from alink_amd import *`` mirrors PyAlink's ``from pyalink.alink import *``: environment helpers
(``useLocalEnv``, ``resetEnv``), every batch/stream operator, pipeline stages, vectors and Params.
"""
__version__ = "0.1.0"

from .common.mlenv import (MLEnvironment, MLEnvironmentFactory, useLocalEnv, useRemoteEnv, resetEnv,  # noqa
                           getMLEnv)
from .common.params import Params, ParamInfo  # noqa: F401
from .parallel.launch import launch, launch_script  # noqa: F401
from .common.linalg import DenseVector, SparseVector, VectorUtil, DenseMatrix, BLAS, MatVecOp, NormalEquation  # noqa: F401,E501
from .common.table import MTable, Row  # noqa: F401
from .common.types import TableSchema, Types  # noqa: F401
from .operator.common.sql.udf import ScalarFunction, TableFunction, udf, udtf  # noqa: F401
from .operator.common.io.db import BaseDB, SqliteDB, DerbyDB, MySqlDB, JdbcDB  # noqa: F401
from .operator.base import BatchOperator  # noqa: F401
from .operator.batch import *  # noqa: F401,F403
from .operator.stream import *  # noqa: F401,F403
from .pipeline import *  # noqa: F401,F403
from .connectors import *  # noqa: F401,F403
from .common.io_registry import IOType, AnnotationUtils, io_op, db_class, register_builtin as _register_io  # noqa

_register_io()

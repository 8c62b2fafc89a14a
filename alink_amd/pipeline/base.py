"""Pipeline API: stages, Trainer, MapTransformer/MapModel, Pipeline, PipelineModel, LocalPredictor.

Reference: ``A/pipeline/{PipelineStageBase,EstimatorBase,TransformerBase,ModelBase,Trainer,MapTransformer,MapModel,
Pipeline,PipelineModel,LocalPredictor,ModelExporterUtils}.java`` and the vendored Flink-ML interfaces
(``F/api/core/*``).

Pipeline-model file format (``ModelExporterUtils.java:40-177``, ``PipelineModel.java:121-151``): one table
``(model_id BIGINT, model_data VARCHAR)``; row ``-1`` holds ``{"clazz":[...],"param":[...],"schema":[...]}``
(JSON arrays of Java class names, stage Params JSON, model-table schema strings); rows with id ``i`` hold
stage ``i``'s model rows, each CSV-encoded with field delimiter ``^`` and quote ``'`` (vectors serialised to
strings first).  Files written here use the Java class names, so Alink can load them and vice versa.
"""
from __future__ import annotations

import json
from typing import Callable, List, Optional, Sequence

from ..common.javafmt import gson_dumps
from ..common.mapper import Mapper, ModelMapper
from ..common.mlenv import MLEnvironmentFactory
from ..common.params import ParamInfo, Params, WithParams
from ..common.table import MTable, Row
from ..common.types import TableSchema, Types, schema_str_to_schema, schema_to_schema_str
from ..operator.base import BatchOperator, gather_table

__all__ = ["ModelExporterUtils", "PipelineStageBase", "EstimatorBase", "TransformerBase", "ModelBase", "Trainer", "MapTransformer",
           "MapModel", "Pipeline", "PipelineModel", "LocalPredictor", "STAGE_REGISTRY", "register_stage",
           "PIPELINE_MODEL_SCHEMA"]

STAGE_REGISTRY = {}
PIPELINE_MODEL_SCHEMA = TableSchema(["model_id", "model_data"], [Types.LONG, Types.STRING])


def register_stage(cls):
    STAGE_REGISTRY[cls.__name__] = cls
    return cls


def java_class_name(cls) -> str:
    from ..params import _spec
    name = getattr(cls, "_ALINK_NAME", cls.__name__)
    info = _spec.OPS.get(name)
    if info is not None:
        p = info["path"]
        pkg = p.split("src/main/java/")[-1][:-len(".java")]
        return pkg.replace("/", ".")
    return "alink_amd." + cls.__module__.split("alink_amd.")[-1] + "." + cls.__name__


def stage_class_from_java(name: str):
    simple = name.split(".")[-1]
    if simple in STAGE_REGISTRY:
        return STAGE_REGISTRY[simple]
    from .. import pipeline as P  # noqa: F401  (registers all stages)
    if simple in STAGE_REGISTRY:
        return STAGE_REGISTRY[simple]
    raise KeyError(f"unknown pipeline stage class {name}")


class PipelineStageBase(WithParams):
    _NO_AUTO_PARAMS = True
    PARAMS = [ParamInfo("MLEnvironmentId", int, "ID of ML environment.", default=0)]

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)

    def getMLEnvironmentId(self):
        return self.getParams().get(PipelineStageBase.PARAMS[0])

    def setMLEnvironmentId(self, v):
        self.getParams().set(PipelineStageBase.PARAMS[0], v)
        return self

    @property
    def env(self):
        return MLEnvironmentFactory.get(self.getMLEnvironmentId())

    def clone(self):
        return type(self)(self.getParams().clone())

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        register_stage(cls)


def _lazy_get(stage, name, default=None):
    p = stage.getParams()
    return p.get(name) if p.contains(name) else default


class _LazyPrintTransformInfo:
    """``HasLazyPrintTransformInfo`` (reference ``common/lazy/HasLazyPrintTransformInfo.java``): the enabled
    flags live in the stage's params, so a model built from a Trainer's params inherits them, and a later
    ``enable*`` on the model overrides what it inherited."""

    def enableLazyPrintTransformData(self, n: int = -1, title: Optional[str] = None):
        p = self.getParams()
        p.set("lazyPrintTransformDataEnabled", True)
        p.set("lazyPrintTransformDataNum", int(n))
        p.set("lazyPrintTransformDataTitle", title)
        return self

    def enableLazyPrintTransformStat(self, title: Optional[str] = None):
        p = self.getParams()
        p.set("lazyPrintTransformStatEnabled", True)
        p.set("lazyPrintTransformStatTitle", title)
        return self


class TransformerBase(_LazyPrintTransformInfo, PipelineStageBase):
    def transform(self, input):
        from ..operator.stream.base import StreamOperator
        if isinstance(input, StreamOperator):
            return self.transformStream(input)
        if isinstance(input, MTable):
            from ..operator.batch.source import TableSourceBatchOp
            input = TableSourceBatchOp(input)
        out = self.transformBatch(input)
        return self._post_process_transform(out)

    def _post_process_transform(self, out):
        """Reference ``TransformerBase.postProcessTransformResult``: record the result, then register the enabled
        lazy prints on it (they fire at the next execution)."""
        self.env.lazy.genLazyTransformResult(self).addValue(out)
        if _lazy_get(self, "lazyPrintTransformDataEnabled", False):
            out.lazyPrint(_lazy_get(self, "lazyPrintTransformDataNum", -1),
                          _lazy_get(self, "lazyPrintTransformDataTitle"))
        if _lazy_get(self, "lazyPrintTransformStatEnabled", False):
            out.lazyPrintStatistics(_lazy_get(self, "lazyPrintTransformStatTitle"))
        return out

    def transformBatch(self, input: BatchOperator) -> BatchOperator:
        raise NotImplementedError

    def transformStream(self, input):
        raise NotImplementedError(f"{type(self).__name__} does not support stream transform")


class ModelBase(TransformerBase):
    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        self.modelData: Optional[MTable] = None

    def getModelData(self) -> MTable:
        return self.modelData

    def setModelData(self, data):
        if isinstance(data, BatchOperator):
            data = data.getOutputTable()
        self.modelData = data
        return self

    def clone(self):
        m = type(self)(self.getParams().clone())
        m.modelData = self.modelData
        return m


class EstimatorBase(PipelineStageBase):
    def fit(self, input) -> ModelBase:
        from ..operator.stream.base import StreamOperator
        if isinstance(input, StreamOperator):
            return self.fitStream(input)
        if isinstance(input, MTable):
            from ..operator.batch.source import TableSourceBatchOp
            input = TableSourceBatchOp(input)
        return self.fitBatch(input)

    def fitBatch(self, input: BatchOperator) -> ModelBase:
        raise NotImplementedError

    def fitStream(self, input):
        raise NotImplementedError("Only support batch fit!")


class Trainer(_LazyPrintTransformInfo, EstimatorBase):
    """``fit = createModel(train(in).getOutputTable())`` (reference ``Trainer.java:33-111``)."""
    TRAIN_OP = None
    MODEL = None

    def train(self, input: BatchOperator) -> BatchOperator:
        return self.TRAIN_OP(self.getParams()).linkFrom(input)

    def createModel(self, model_table: MTable) -> ModelBase:
        model_cls = self.MODEL if not isinstance(self.MODEL, str) else STAGE_REGISTRY[self.MODEL]
        return model_cls(self.getParams().clone()).setModelData(model_table)

    def fitBatch(self, input):
        op = self.train(input)
        lm = self.env.lazy
        # postProcessTrainOp: record the train op and register the enabled train / model info prints on it
        lm.genLazyTrainOp(self).addValue(op)
        if _lazy_get(self, "lazyPrintTrainInfoEnabled", False) and hasattr(op, "lazyPrintTrainInfo"):
            op.lazyPrintTrainInfo(_lazy_get(self, "lazyPrintTrainInfoTitle"))
        if _lazy_get(self, "lazyPrintModelInfoEnabled", False) and hasattr(op, "lazyPrintModelInfo"):
            op.lazyPrintModelInfo(_lazy_get(self, "lazyPrintModelInfoTitle"))
        # postProcessModel: the model is built from this trainer's params, so it inherits the transform flags
        model = self.createModel(op.getOutputTable())
        lm.genLazyModel(self).addValue(model)
        self._train_op = op
        return model

    # HasLazyPrintTrainInfo / HasLazyPrintModelInfo: flags in params, applied to the train op of each fit
    def enableLazyPrintTrainInfo(self, title: Optional[str] = None):
        self.getParams().set("lazyPrintTrainInfoEnabled", True)
        self.getParams().set("lazyPrintTrainInfoTitle", title)
        return self

    def enableLazyPrintModelInfo(self, title: Optional[str] = None):
        self.getParams().set("lazyPrintModelInfoEnabled", True)
        self.getParams().set("lazyPrintModelInfoTitle", title)
        return self


class MapTransformer(TransformerBase):
    MAPPER: Callable[..., Mapper] = None

    def transformBatch(self, input):
        from ..operator.batch.utils import MapBatchOp
        return MapBatchOp(self.getParams(), mapper=self.MAPPER).linkFrom(input)

    def transformStream(self, input):
        from ..operator.stream.base import MapStreamOp
        return MapStreamOp(self.getParams(), mapper=self.MAPPER).linkFrom(input)

    def getLocalPredictor(self, inputSchema):
        if isinstance(inputSchema, str):
            inputSchema = schema_str_to_schema(inputSchema)
        return LocalPredictor(self.MAPPER(inputSchema, self.getParams()))


class MapModel(ModelBase):
    MAPPER: Callable[..., ModelMapper] = None

    def transformBatch(self, input):
        from ..operator.batch.source import TableSourceBatchOp
        from ..operator.batch.utils import ModelMapBatchOp
        return ModelMapBatchOp(self.getParams(), mapper=self.MAPPER).linkFrom(
            TableSourceBatchOp(self.getModelData()), input)

    def transformStream(self, input):
        from ..operator.batch.source import TableSourceBatchOp
        from ..operator.stream.base import ModelMapStreamOp
        return ModelMapStreamOp(TableSourceBatchOp(self.getModelData()), self.getParams(),
                                mapper=self.MAPPER).linkFrom(input)

    def getLocalPredictor(self, inputSchema):
        if isinstance(inputSchema, str):
            inputSchema = schema_str_to_schema(inputSchema)
        full = gather_table(self.getModelData())
        m = self.MAPPER(full.schema, inputSchema, self.getParams())
        m.loadModel(full.rows())
        m.open()
        return LocalPredictor(m)


class LocalPredictor:
    """Row-at-a-time serving chain (reference ``LocalPredictor.java:18-62``)."""

    def __init__(self, *mappers):
        self.mappers: List[Mapper] = list(mappers)

    def merge(self, other: "LocalPredictor"):
        self.mappers.extend(other.mappers)
        return self

    def getOutputSchema(self) -> TableSchema:
        return self.mappers[-1].getOutputSchema()

    def map(self, row) -> Row:
        r = tuple(row)
        for m in self.mappers:
            r = m.map(r)
        return Row(r)

    def map_batch(self, rows) -> List[Row]:
        """Batched serving: runs each mapper's columnar path once over all rows."""
        mt = MTable.from_rows([tuple(r) for r in rows], self.mappers[0].getDataSchema())
        for m in self.mappers:
            mt = m.map_table(mt)
        return mt.rows()

    def close(self):
        for m in self.mappers:
            m.close()


class Pipeline(EstimatorBase):
    def __init__(self, *stages, params: Optional[Params] = None):
        super().__init__(params)
        if len(stages) == 1 and isinstance(stages[0], (list, tuple)):
            stages = stages[0]
        self.stages: List[PipelineStageBase] = list(stages)

    def add(self, *args):
        if len(args) == 2 and isinstance(args[0], int):
            self.stages.insert(args[0], args[1])
        else:
            self.stages.extend(args)
        return self

    def remove(self, index: int):
        return self.stages.pop(index)

    def get(self, index: int):
        return self.stages[index]

    def size(self):
        return len(self.stages)

    def _last_estimator(self):
        last = -1
        for i, s in enumerate(self.stages):
            if isinstance(s, EstimatorBase):
                last = i
        return last

    def fitBatch(self, input):
        last = self._last_estimator()
        transformers = []
        for i, s in enumerate(self.stages):
            if i <= last:
                if isinstance(s, EstimatorBase):
                    t = s.fit(input)
                else:
                    t = s
                if i < last:
                    input = t.transform(input)
            else:
                t = s
            transformers.append(t)
        return PipelineModel(transformers).setMLEnvironmentId(self.getMLEnvironmentId())

    def fitStream(self, input):
        last = self._last_estimator()
        if last >= 0:
            raise RuntimeError("Pipeline with estimators can not be fit on a stream")
        return PipelineModel(list(self.stages))


class PipelineModel(ModelBase):
    def __init__(self, *transformers, params: Optional[Params] = None):
        if len(transformers) == 1 and isinstance(transformers[0], Params):
            params, transformers = transformers[0], ()
        super().__init__(params)
        if len(transformers) == 1 and isinstance(transformers[0], (list, tuple)):
            transformers = transformers[0]
        self.transformers: List[TransformerBase] = list(transformers)

    def getTransformers(self) -> List[TransformerBase]:
        return list(self.transformers)

    def getTransformer(self, i: int) -> TransformerBase:
        return self.transformers[i]

    def transformBatch(self, input):
        for t in self.transformers:
            input = t.transform(input)
        return input

    def transformStream(self, input):
        for t in self.transformers:
            input = t.transform(input)
        return input

    def getLocalPredictor(self, inputSchema):
        if isinstance(inputSchema, str):
            inputSchema = schema_str_to_schema(inputSchema)
        if not self.transformers:
            raise RuntimeError("PipelineModel is empty.")
        pred = None
        schema = inputSchema
        for t in self.transformers:
            if not hasattr(t, "getLocalPredictor"):
                raise RuntimeError(f"{type(t)} not support local predict.")
            lp = t.getLocalPredictor(schema)
            schema = lp.getOutputSchema()
            pred = lp if pred is None else pred.merge(lp)
        return pred

    # ---- persistence ----
    def save(self, path: Optional[str] = None, overwrite: bool = True):
        op = pack_transformers(self.transformers)
        if path is None:
            return op
        from ..operator.batch.sink import CsvSinkBatchOp
        op.link(CsvSinkBatchOp().setFilePath(path).setOverwriteSink(overwrite))
        return op

    @staticmethod
    def load(src) -> "PipelineModel":
        if isinstance(src, str):
            from ..operator.batch.source import CsvSourceBatchOp
            src = CsvSourceBatchOp().setFilePath(src).setSchemaStr("model_id bigint, model_data string")
        rows = src.collect() if isinstance(src, BatchOperator) else list(src)
        return PipelineModel(unpack_transformers(rows))

    @staticmethod
    def collectLoad(src):
        return PipelineModel.load(src)


def _model_rows_as_strings(mt: MTable) -> (List[str], TableSchema):
    from ..common.linalg import Vector, VectorUtil
    from ..common.types import is_vector
    from ..operator.common.io.csv import CsvFormatter
    full = gather_table(mt)
    types = [Types.STRING if is_vector(t) else t for t in full.schema.types]
    schema = TableSchema(full.schema.names, types)
    fmt = CsvFormatter(types, "^", "'")
    out = []
    for r in full.rows():
        rr = [VectorUtil.toString(v) if isinstance(v, Vector) else v for v in r]
        out.append(fmt.format(rr))
    return out, schema


def pack_rows(transformers: Sequence[TransformerBase]) -> List[Row]:
    clazz, params, schemas = [], [], []
    payload = []
    for i, t in enumerate(transformers):
        clazz.append(java_class_name(type(t)))
        params.append(t.getParams().toJson())
        if isinstance(t, PipelineModel):
            schemas.append(schema_to_schema_str(PIPELINE_MODEL_SCHEMA))
            sub = pack_rows(t.transformers)
            from ..operator.common.io.csv import CsvFormatter
            fmt = CsvFormatter([Types.LONG, Types.STRING], "^", "'")
            payload.extend(Row((i, fmt.format(r))) for r in sub)
        elif isinstance(t, ModelBase) and t.modelData is not None:
            lines, schema = _model_rows_as_strings(t.modelData)
            schemas.append(schema_to_schema_str(schema))
            payload.extend(Row((i, l)) for l in lines)
        else:
            schemas.append("")
    config = gson_dumps({"clazz": clazz, "param": params, "schema": schemas}, java_map_order=True)
    return [Row((-1, config))] + payload


def pack_transformers(transformers) -> BatchOperator:
    from ..operator.batch.source import MemSourceBatchOp
    return MemSourceBatchOp(pack_rows(transformers), PIPELINE_MODEL_SCHEMA)


def unpack_transformers(rows) -> List[TransformerBase]:
    from ..operator.common.io.csv import CsvParser
    rows = [tuple(r) for r in rows]
    conf = [r for r in rows if int(r[0]) == -1]
    if len(conf) != 1:
        raise ValueError("Invalid model.")
    cfg = json.loads(conf[0][1])
    out = []
    for i, (cz, ps, sc) in enumerate(zip(cfg["clazz"], cfg["param"], cfg["schema"])):
        cls = stage_class_from_java(cz)
        p = Params.fromJson(ps)
        data_lines = [r[1] for r in rows if int(r[0]) == i]
        if cls is PipelineModel:
            parser = CsvParser([Types.LONG, Types.STRING], "^", "'")
            sub = [parser.parse(l)[1] for l in data_lines]
            out.append(PipelineModel(unpack_transformers(sub)))
            continue
        t = cls(p)
        if isinstance(t, ModelBase) and sc:
            schema = schema_str_to_schema(sc)
            parser = CsvParser(schema.types, "^", "'")
            mrows = [parser.parse(l)[1] for l in data_lines]
            t.setModelData(MTable.from_rows(mrows, schema, replicated=True))
        out.append(t)
    return out


class ModelExporterUtils:
    """``ModelExporterUtils.java`` — pack pipeline stages into / unpack them from the one-table pipeline model
    format (``(model_id, model_data)`` with the ``-1`` config row and ``^``-delimited per-stage rows)."""
    packTransformersArray = staticmethod(pack_transformers)
    packRows = staticmethod(pack_rows)
    unpackTransformersArray = staticmethod(unpack_transformers)

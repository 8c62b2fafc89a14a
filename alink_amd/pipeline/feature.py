"""Feature / data-processing pipeline stages (reference ``A/pipeline/{dataproc,feature}/*``)."""
from ..models.feature import encoders as E
from ..models.feature import scalers as S
from ..operator.batch import feature as F
from .base import MapModel, MapTransformer, Trainer

__all__ = []


def _stage(name, base, **attrs):
    cls = type(name, (base,), dict(attrs, __module__=__name__))
    globals()[name] = cls
    __all__.append(name)
    return cls


for _n, _mapper in (("StandardScaler", S.StandardScalerModelMapper), ("MinMaxScaler", S.MinMaxScalerModelMapper),
                    ("MaxAbsScaler", S.MaxAbsScalerModelMapper), ("Imputer", S.ImputerModelMapper),
                    ("VectorStandardScaler", S.VectorScalerModelMapper),
                    ("VectorMinMaxScaler", S.VectorScalerModelMapper),
                    ("VectorMaxAbsScaler", S.VectorScalerModelMapper),
                    ("VectorImputer", S.VectorImputerModelMapper),
                    ("StringIndexer", E.StringIndexerModelMapper),
                    ("MultiStringIndexer", E.MultiStringIndexerModelMapper),
                    ("QuantileDiscretizer", E.QuantileDiscretizerModelMapper)):
    _stage(_n + "Model", MapModel, MAPPER=_mapper)
    _stage(_n, Trainer, TRAIN_OP=getattr(F, _n + "TrainBatchOp"), MODEL=_n + "Model")

_stage("OneHotEncoderModel", MapModel, MAPPER=E.OneHotModelMapper)
_stage("OneHotEncoder", Trainer, TRAIN_OP=F.OneHotTrainBatchOp, MODEL="OneHotEncoderModel")
_stage("IndexToString", MapModel, MAPPER=E.IndexToStringModelMapper)

# StringIndexerModel.registeredModel: a model fitted with ``modelName`` is found by name from IndexToString
# (reference pipeline/dataproc/StringIndexerModel.java:20-50, IndexToString.java:66-72)
_REGISTERED_STRING_INDEXERS: dict = {}


def _model_name(stage):
    p = stage.getParams()
    try:
        return p.get("modelName") if p.contains("modelName") else None
    except KeyError:
        return None


def _register_string_indexer(self, data):
    MapModel.setModelData(self, data)
    name = _model_name(self)
    if name is not None:
        _REGISTERED_STRING_INDEXERS[name] = self
    return self


def _index_to_string_model_data(self):
    if self.modelData is None:
        name = _model_name(self)
        if name not in _REGISTERED_STRING_INDEXERS:
            raise ValueError(f"Can't find StringIndexerModel with name: {name}")
        self.setModelData(_REGISTERED_STRING_INDEXERS[name].getModelData())
    return self.modelData


StringIndexerModel.setModelData = _register_string_indexer          # noqa: F821 (defined by _stage)
IndexToString.getModelData = _index_to_string_model_data            # noqa: F821
_stage("Binarizer", MapTransformer, MAPPER=E.BinarizerMapper)
_stage("Bucketizer", MapTransformer, MAPPER=E.BucketizerMapper)
_stage("FeatureHasher", MapTransformer, MAPPER=E.FeatureHasherMapper)
_stage("DCT", MapTransformer, MAPPER=E.DCTMapper)

from ..models.feature import pca as _PCA  # noqa: E402
_stage("PCAModel", MapModel, MAPPER=_PCA.PcaModelMapper)
_stage("PCA", Trainer, TRAIN_OP=F.PcaTrainBatchOp, MODEL="PCAModel")

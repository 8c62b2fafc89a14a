"""Pipeline stages of the non-linear classifiers (reference ``A/pipeline/classification/*``)."""
from ..models.classification.naive_bayes import NaiveBayesTextModelMapper
from ..operator.batch import classification_extra as C
from .base import MapModel, Trainer

__all__ = ["OneVsRest", "OneVsRestModel", "FmClassifier", "FmRegressor", "FmModel", "NaiveBayesTextClassifier", "NaiveBayesTextModel", "MultilayerPerceptronClassifier",
           "MultilayerPerceptronClassificationModel"]


class NaiveBayesTextClassifier(Trainer):
    TRAIN_OP = C.NaiveBayesTextTrainBatchOp
    MODEL = "NaiveBayesTextModel"


class NaiveBayesTextModel(MapModel):
    MAPPER = NaiveBayesTextModelMapper


from ..models.classification.mlp import MlpcModelMapper  # noqa: E402


class MultilayerPerceptronClassifier(Trainer):
    TRAIN_OP = C.MultilayerPerceptronTrainBatchOp
    MODEL = "MultilayerPerceptronClassificationModel"


class MultilayerPerceptronClassificationModel(MapModel):
    MAPPER = MlpcModelMapper


from ..models.recommendation.fm import FmModelMapper  # noqa: E402


class FmClassifier(Trainer):
    TRAIN_OP = C.FmClassifierTrainBatchOp
    MODEL = "FmModel"


class FmRegressor(Trainer):
    TRAIN_OP = C.FmRegressorTrainBatchOp
    MODEL = "FmModel"


class FmModel(MapModel):
    MAPPER = FmModelMapper


from ..models.classification.onevsrest import OneVsRestModelMapper, build_ovr_model_table  # noqa: E402
from .base import EstimatorBase, java_class_name  # noqa: E402


class OneVsRestModel(MapModel):
    MAPPER = OneVsRestModelMapper


class OneVsRest(EstimatorBase):
    """Train ``numClass`` binary copies of ``classifier`` (class i vs rest) — ``OneVsRest.java``."""
    _NO_AUTO_PARAMS = False

    def __init__(self, params=None, **kw):
        super().__init__(params, **kw)
        self.classifier = None

    def setClassifier(self, c):
        self.classifier = c
        return self

    def getClassifier(self):
        return self.classifier

    def fitBatch(self, input):
        from ..common.types import Types
        from ..operator.base import gather_table
        from ..operator.batch.source import TableSourceBatchOp
        mt = input.getOutputTable()
        label_col = self.classifier.getParams().get("labelCol")
        lt = mt.col_type(label_col)
        from ..parallel import comm
        distinct = set()
        for part in comm.all_gather_object(list(set(mt.col(label_col).to_list()))):
            distinct.update(part)
        labels = sorted(distinct)
        n = int(self.get("numClass"))
        if n > len(labels):
            raise RuntimeError("the specified numClasses is larger than the number of distinct labels.")
        li = mt.col_index(label_col)
        models = []
        for i in range(n):
            target = labels[i]
            vals = [1.0 if v == target else 0.0 for v in mt.col(label_col).to_list()]
            names = list(mt.schema.names)
            types = list(mt.schema.types)
            types[li] = Types.DOUBLE
            cols = list(mt.cols)
            from ..common.table import Column
            cols[li] = Column.from_values(vals, Types.DOUBLE)
            from ..common.table import MTable as _MT
            from ..common.types import TableSchema as _TS
            sub = _MT(_TS(names, types), cols, mt.replicated)
            clf = self.classifier.clone()
            clf.getParams().set("positiveLabelValueString", "1")
            models.append(gather_table(clf.fit(TableSourceBatchOp(sub)).getModelData()))
        table = build_ovr_model_table(models, labels[:n] if n < len(labels) else labels, lt,
                                      java_class_name(type(self.classifier)), self.classifier.getParams(), n)
        p = self.classifier.getParams().clone().merge(self.getParams())
        return OneVsRestModel(p).setModelData(table)

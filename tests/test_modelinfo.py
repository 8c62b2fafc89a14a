"""ExtractModelInfoBatchOp / WithModelInfoBatchOp (A/common/lazy/*) with the FM model summary
(A/operator/common/fm/FmModelInfo.java): eager collect, lazy callbacks firing on collect, printed text."""
import numpy as np

from alink_amd import useLocalEnv, FmRegressorTrainBatchOp, FmModelInfoBatchOp
from alink_amd.operator.batch.source import MemSourceBatchOp


def _train():
    useLocalEnv(1, device="cpu")
    rng = np.random.default_rng(0)
    rows = [[float(a), float(b), float(2 * a - b + 0.1 * c)] for a, b, c in rng.normal(size=(200, 3))]
    src = MemSourceBatchOp(rows, "f0 double, f1 double, label double")
    return FmRegressorTrainBatchOp().setFeatureCols(["f0", "f1"]).setLabelCol("label").setNumFactor(4) \
        .setNumEpochs(3).linkFrom(src)


def test_fm_model_info_collect():
    op = _train()
    info = op.collectModelInfo()
    assert info.getTask() == "REGRESSION"
    assert info.getDim()[2] == 4
    assert info.getFactors().shape == (2, 4)
    assert info.getColNames() == ["f0", "f1"]
    text = str(info)
    assert "meta info" in text and "model info" in text and "f0" in text


def test_fm_model_info_lazy(capsys):
    op = _train()
    got = []
    op.lazyCollectModelInfo(lambda i: got.append(i.getVectorSize()))
    op.lazyPrintModelInfo("FM summary")
    op.collect()
    assert got == [2]
    assert "FM summary" in capsys.readouterr().out


def test_extract_op_passes_model_through():
    op = _train()
    ex = FmModelInfoBatchOp().linkFrom(op)
    assert ex.collect() == op.collect()

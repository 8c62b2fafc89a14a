"""Lazy printing on pipeline stages (reference tier-5 suite ``core/src/test/java/com/alibaba/alink/common/lazy/
PipelineLazyTest.java``, ``TrainModelInfoTest.java``): the ``enableLazyPrint*`` flags of trainers and models fire
at the next execution, models inherit a trainer's transform flags, and a model's own setting overrides them.
The reference runs these on fake operators; here a real LogisticRegression trainer / model plays their part."""
import pandas as pd
import pytest

from alink_amd import BatchOperator, LogisticRegression, MLEnvironmentFactory, useLocalEnv

COLS = ["label", "u", "i", "r"]


@pytest.fixture(autouse=True)
def _env():
    useLocalEnv(1)
    yield


def _src(cols=COLS, env_id=None):
    df = pd.DataFrame({"label": [0, 1, 0, 1, 1, 0, 1, 0], "u": [1.0, 2.0, 1.5, 3.0, 2.5, 0.5, 3.5, 1.0],
                       "i": [0.1, 0.9, 0.2, 0.8, 0.7, 0.3, 0.6, 0.1], "r": [1.0, 5.0, 2.0, 4.0, 4.0, 1.0, 5.0, 2.0]})
    df.columns = cols
    op = BatchOperator.fromDataframe(df, schemaStr=", ".join(f"{c} {'int' if c == 'label' else 'double'}"
                                                              for c in cols))
    return op if env_id is None else op.setMLEnvironmentId(env_id)


def _trainer(cols=COLS):
    return LogisticRegression().setFeatureCols(cols[1:]).setLabelCol("label").setPredictionCol("pred") \
        .setMaxIter(5)


def test_trainer_prints_model_train_info_and_transform_data_stat(capsys):
    src = _src()
    t = _trainer()
    t.enableLazyPrintModelInfo("===== MODEL INFO =====")
    t.enableLazyPrintTrainInfo("===== TRAIN INFO =====")
    t.enableLazyPrintTransformStat("===== TRAINER TRANSFORM STAT =====")
    t.enableLazyPrintTransformData(5, "===== TRAINER TRANSFORM DATA =====")
    model = t.fit(src)
    model.transform(src).firstN(5).print()
    out = capsys.readouterr().out
    for title in ("===== MODEL INFO =====", "===== TRAIN INFO =====", "===== TRAINER TRANSFORM STAT =====",
                  "===== TRAINER TRANSFORM DATA ====="):
        assert title in out, title
    assert "|".join(src.getColNames()) in out.replace(" ", "")
    for word in ("count", "numMissingValue", "normL1", "normL2"):
        assert word in out, word


def test_transformer_flags_on_the_model(capsys):
    src = _src()
    model = _trainer().fit(src)
    model.enableLazyPrintTransformData(5, "===== TRANSFORM DATA =====")
    model.enableLazyPrintTransformStat("===== TRANSFORM STAT =====")
    model.transform(src).firstN(5).print()
    out = capsys.readouterr().out
    assert "===== TRANSFORM DATA =====" in out and "===== TRANSFORM STAT =====" in out
    assert "normL2" in out


def test_trainer_without_fit_prints_nothing(capsys):
    title = "===== LAZY PRINT CALLBACK ===="
    src = _src()
    t = _trainer()
    t.enableLazyPrintTrainInfo(title)
    src.print()
    assert title not in capsys.readouterr().out
    t.fit(src).transform(src).print()
    assert title in capsys.readouterr().out


def test_model_flag_fires_for_every_transform(capsys):
    title = "===== LAZY PRINT CALLBACK ====="
    model = _trainer().fit(_src())
    model.enableLazyPrintTransformStat(title)
    model.transform(_src())
    model.transform(_src()).print()
    assert capsys.readouterr().out.count(title) == 2


def test_trainer_flag_is_inherited_by_every_model(capsys):
    title = "===== LAZY PRINT CALLBACK ====="
    t = _trainer()
    t.enableLazyPrintTransformStat(title)
    m1, m2 = t.fit(_src()), t.fit(_src())
    outs = [m.transform(_src()) for m in (m1, m1, m2, m2)]
    outs[0].print()
    assert capsys.readouterr().out.count(title) == 4


def test_model_setting_overrides_the_inherited_one(capsys):
    title, title2 = "===== LAZY PRINT CALLBACK =====", "===== LAZY PRINT CALLBACK2 ====="
    t = _trainer()
    t.enableLazyPrintTransformStat(title)
    m1, m2 = t.fit(_src()), t.fit(_src())
    m1.enableLazyPrintTransformStat(title2)
    outs = [m.transform(_src()) for m in (m1, m1, m2, m2)]
    outs[0].print()
    out = capsys.readouterr().out
    assert out.count(title) == 2 and out.count(title2) == 2


def test_non_default_environment(capsys):
    env_id = MLEnvironmentFactory.getNewMLEnvironmentId()
    try:
        src = _src(env_id=env_id)
        t = _trainer().setMLEnvironmentId(env_id)
        t.enableLazyPrintModelInfo("===== MODEL INFO =====")
        t.enableLazyPrintTransformStat("===== TRAINER TRANSFORM STAT =====")
        model = t.fit(src)
        model.transform(src).firstN(5).print()
    finally:
        MLEnvironmentFactory.remove(env_id)
    out = capsys.readouterr().out
    assert "===== MODEL INFO =====" in out and "===== TRAINER TRANSFORM STAT =====" in out


# ---- BatchOperator lazy sinks (reference BatchOperatorLazyTest.java) ----
ROWS = [(1, 1, 0.6), (2, 2, 0.8), (2, 3, 0.6), (4, 1, 0.6), (4, 2, 0.3), (4, 3, 0.4)]


def _mem(cols, env_id=None):
    from alink_amd import MemSourceBatchOp
    op = MemSourceBatchOp(ROWS, cols)
    return op if env_id is None else op.setMLEnvironmentId(env_id)


def _header(cols):
    return "|".join(cols)


def test_lazy_print_fires_in_execute(capsys):
    _mem(["u", "i", "r"]).lazyPrint(-1, "This is table 1")
    _mem(["uu", "ii", "rr"]).lazyPrint(-1, "This is table 2")
    BatchOperator.execute()
    out = capsys.readouterr().out
    assert "This is table 1" in out and "This is table 2" in out


def test_lazy_print_fires_in_collect_and_print(capsys):
    a, b = _mem(["u", "i", "r"]), _mem(["uu", "ii", "rr"])
    a.lazyPrint(-1)
    b.lazyPrint(-1)
    assert len(_mem(["uuu", "iii", "rrr"]).collect()) == len(ROWS)
    out = capsys.readouterr().out.replace(" ", "")
    assert _header(a.getColNames()) in out and _header(b.getColNames()) in out
    a.lazyPrint(-1)
    _mem(["uuu", "iii", "rrr"]).print()
    out = capsys.readouterr().out.replace(" ", "")
    assert _header(a.getColNames()) in out and _header(["uuu", "iii", "rrr"]) in out


def test_lazy_collect_callbacks_in_print(capsys):
    got = []
    _mem(["u", "i", "r"]).lazyCollect(lambda d: got.append(("cb1", len(d))), lambda d: got.append(("cb2", len(d))))
    _mem(["uu", "ii", "rr"]).lazyPrint(-1)
    _mem(["uuu", "iii", "rrr"]).print()
    assert got == [("cb1", len(ROWS)), ("cb2", len(ROWS))]
    assert _header(["uu", "ii", "rr"]) in capsys.readouterr().out.replace(" ", "")


def test_exception_in_lazy_collect_propagates():
    def boom(_):
        raise AssertionError("callback failed")
    _mem(["u", "i", "r"]).lazyCollect(lambda d: None, boom)
    with pytest.raises(AssertionError):
        BatchOperator.execute()


def test_lazy_statistics(capsys):
    _mem(["u", "i", "r"]).lazyPrintStatistics("==== TITLE ====")
    BatchOperator.execute()
    out = capsys.readouterr().out
    for word in ("==== TITLE ====", "numMissingValue", "count", "normL1", "normL2"):
        assert word in out, word


def test_sinks_fire_once(capsys):
    from alink_amd import FirstNBatchOp
    a = _mem(["label", "u", "i"])
    a.lazyPrint(-1, "This is table 1")
    BatchOperator.execute()
    assert "This is table 1" in capsys.readouterr().out
    _mem(["label", "u", "i"]).print()
    assert "This is table 1" not in capsys.readouterr().out
    b = _mem(["label", "u", "i"])
    b.lazyPrint(-1, "This is table 2")
    FirstNBatchOp().setSize(10).linkFrom(b).print()
    assert "This is table 2" in capsys.readouterr().out
    FirstNBatchOp().setSize(10).linkFrom(b).print()
    assert "This is table 2" not in capsys.readouterr().out


def test_lazy_print_in_non_default_env(capsys):
    env_id = MLEnvironmentFactory.getNewMLEnvironmentId()
    try:
        _mem(["u", "i", "r"], env_id).lazyPrint(-1, "This is table 1")
        _mem(["uu", "ii", "rr"], env_id).lazyPrint(-1, "This is table 2")
        BatchOperator.execute(MLEnvironmentFactory.get(env_id))
    finally:
        MLEnvironmentFactory.remove(env_id)
    out = capsys.readouterr().out
    assert "This is table 1" in out and "This is table 2" in out


# ---- train / model info (reference TrainModelInfoTest.java) and LazyEvaluation (LazyEvaluationTest.java) ----
def _lr_op(env_id=None):
    from alink_amd import LogisticRegressionTrainBatchOp
    op = LogisticRegressionTrainBatchOp().setFeatureCols(["u", "i", "r"]).setLabelCol("label").setMaxIter(5)
    if env_id is not None:
        op.setMLEnvironmentId(env_id)
    return op.linkFrom(_src(env_id=env_id))


def test_train_and_model_info_collect():
    op = _lr_op()
    assert str(op.collectTrainInfo()).startswith("numIter: ")
    assert str(op.collectModelInfo()).startswith("model: Logistic Regression, intercept: True, coef: ")


def test_lazy_train_and_model_info_fire_on_execute(capsys):
    env_id = MLEnvironmentFactory.getNewMLEnvironmentId()
    try:
        op = _lr_op(env_id)
        got = []
        op.lazyCollectModelInfo(lambda d: got.append(("model", str(d))))
        op.lazyCollectTrainInfo(lambda d: got.append(("train", d.numIter)))
        op.lazyPrintTrainInfo("======= TRAIN INFO =======")
        assert got == [] and "TRAIN INFO" not in capsys.readouterr().out      # nothing before the execution
        BatchOperator.execute(MLEnvironmentFactory.get(env_id))
    finally:
        MLEnvironmentFactory.remove(env_id)
    assert [k for k, _ in got] == ["model", "train"] and got[1][1] >= 1
    out = capsys.readouterr().out
    assert "======= TRAIN INFO =======" in out and "numIter: " in out


def test_lazy_evaluation_values_and_callbacks():
    from alink_amd.common.lazy import LazyEvaluation
    seen = []
    lz = LazyEvaluation()
    lz.addCallback(lambda d: seen.append(d - 1))
    for v in (100, 300, 400):
        lz.addValue(v)
    lz.addCallback(lambda d: seen.append(d + 1))
    lz.addValue(200)
    lz.addCallback(lambda d: seen.append(d + 2))
    assert lz.getLatestValue() == 200
    assert len(seen) == 12                        # 4 values x 3 callbacks
    with pytest.raises(RuntimeError):
        LazyEvaluation().getLatestValue()
    bad = LazyEvaluation()
    bad.addCallback(lambda d: (_ for _ in ()).throw(ValueError("callback failed")))
    with pytest.raises(ValueError):
        bad.addValue(1)

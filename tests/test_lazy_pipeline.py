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

"""DirectReader policies, DataBridge and ModelSource (reference DirectReader.java:61-190, *ModelSource.java)."""
import os

import pytest

from alink_amd.common.directreader import (BroadcastModelSource, DataBridgeModelSource, DirectReader,
                                           DirectReaderPropertiesStore, MemoryDataBridge, DbDataBridge,
                                           DummyDataBridge, RowsModelSource, register_data_bridge,
                                           DataBridgeGenerator)


@pytest.fixture(autouse=True)
def _clean_props():
    DirectReaderPropertiesStore.clear()
    yield
    DirectReaderPropertiesStore.clear()


def _model():
    from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
    useLocalEnv(1)
    src = RandomVectorSourceBatchOp().setNumRows(300).setSize(4).setNumClusters(3).setOutputCol("vec")
    return src, KMeansTrainBatchOp().setVectorCol("vec").setK(3).setMaxIter(5).linkFrom(src)


def test_policies_memory_db_dummy(tmp_path):
    _, model = _model()
    ref = [list(r) for r in model.collect()]
    b = DirectReader.collect(model)
    assert isinstance(b, MemoryDataBridge)
    assert [list(r) for r in DirectReader.directRead(b)] == ref
    DirectReaderPropertiesStore.setProperties({"direct.reader.policy": "db",
                                               "direct.reader.db.path": str(tmp_path / "bridge.sqlite")})
    b = DirectReader.collect(model)
    assert isinstance(b, DbDataBridge)
    assert sorted(map(str, (list(r) for r in b.read()))) == sorted(map(str, ref))
    first = b.read(filter=lambda r: r[0] == 0)
    assert len(first) == 1
    DirectReaderPropertiesStore.setProperties({"direct.reader.policy": "dummy"})
    assert isinstance(DirectReader.collect(model), DummyDataBridge)
    assert DirectReader.collect(model).read() == []


def test_policy_resolution_order(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / "direct_reader.properties").write_text("# comment\ndirect.reader.policy = dummy\n")
    assert DirectReader.policy() == "dummy"
    monkeypatch.setenv("ALINK_DIRECT_READER_POLICY", "db")
    assert DirectReader.policy() == "db"
    DirectReaderPropertiesStore.setProperties({"direct.reader.policy": "memory"})
    assert DirectReader.policy() == "memory"


def test_unknown_policy_and_plugin_registration():
    _, model = _model()
    DirectReaderPropertiesStore.setProperties({"direct.reader.policy": "nope"})
    with pytest.raises(ValueError):
        DirectReader.collect(model)

    @register_data_bridge("firstrow")
    class FirstRow(DataBridgeGenerator):
        def generate(self, op, props):
            mt = op.getOutputTable()
            return MemoryDataBridge(mt.rows()[:1], mt.schema)

    DirectReaderPropertiesStore.setProperties({"direct.reader.policy": "FirstRow"})
    assert len(DirectReader.collect(model).read()) == 1


def test_model_sources_equivalent_for_prediction():
    from alink_amd.operator.batch.utils import load_model_mapper
    from alink_amd.models.clustering.kmeans import KMeansModelMapper
    from alink_amd.common.params import Params
    src, model = _model()
    data = src.getOutputTable()
    p = Params().set("predictionCol", "pred")
    outs = []
    mt = model.getOutputTable()
    for ms in (BroadcastModelSource(mt), RowsModelSource(mt.rows(), mt.schema),
               DataBridgeModelSource(DirectReader.collect(model)), mt):
        m = load_model_mapper(KMeansModelMapper, ms, data.schema, p)
        outs.append([r[-1] for r in m.map_table(data).rows()])
    assert all(o == outs[0] for o in outs)


def test_stream_predict_uses_configured_bridge(tmp_path):
    from alink_amd import KMeansPredictStreamOp, StreamOperator
    from alink_amd.operator.stream.utils import CollectStreamOp
    from alink_amd.operator.stream.source import TableSourceStreamOp
    src, model = _model()
    DirectReaderPropertiesStore.setProperties({"direct.reader.policy": "db",
                                               "direct.reader.db.path": str(tmp_path / "b.sqlite")})
    pred = KMeansPredictStreamOp(model).setPredictionCol("pred").linkFrom(TableSourceStreamOp(src.getOutputTable()))
    assert isinstance(pred._bridge, DbDataBridge)
    box = []
    pred.link(CollectStreamOp(box))
    StreamOperator.execute()
    got = [r[-1] for r in box]
    from alink_amd import KMeansPredictBatchOp
    ref = [r[-1] for r in KMeansPredictBatchOp().setPredictionCol("pred").linkFrom(model, src).collect()]
    assert sorted(got) == sorted(ref)

"""LDA (em / online) on the reference docs corpus (docs/en/ldatrainbatchop.md)."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import *  # noqa: F401,F403

DOCS = ["a b b c c c c c c e e f f f g h k k k", "a b b b d e e e h h k", "a b b b b c f f f f g g g g g g g g g i j j",
        "a a b d d d g g g g g i i j j j k k k k k k k k k", "a a a b c d d d d d d d d d e e e g g j k k k",
        "a a a a b b d d d e e e e f f f f f g h i j j j j", "a a b d d d g g g g g i i j j k k k k k k k k k",
        "a b c d d d d d d d d d e e f g g j k k k", "a a a a b b b b d d d e e e e f f g h h h",
        "a a b b b b b b b b c c e e e g g i i j j j j j j j k k", "a b c d d d d d d d d d f f g g j j j k k k",
        "a a a a b e e e e f f f f f g h h h j"]


@pytest.mark.parametrize("method", ["em", "online"])
def test_lda_doc_corpus(method):
    src = BatchOperator.fromDataframe(pd.DataFrame({"doc": DOCS}), schemaStr="doc string")
    train = LdaTrainBatchOp().setSelectedCol("doc").setTopicNum(6 if method == "em" else 5).setMethod(method) \
        .setSubsamplingRate(1.0).setOptimizeDocConcentration(True).setNumIter(50)
    model = train.linkFrom(src)
    rows = model.collect()
    meta = json.loads(rows[0][1])
    K = 6 if method == "em" else 5
    assert json.loads(meta["topicNum"]) == K and json.loads(meta["vocabularySize"]) == 11
    assert json.loads(meta["method"]) == method
    ll, lp = float(meta["logLikelihood"]), float(meta["logPerplexity"])
    assert ll < 0 and lp == pytest.approx(-ll / sum(len(d.split()) for d in DOCS))
    mat = json.loads(rows[1][1])
    assert (mat["m"], mat["n"]) == ((12, K) if method == "em" else (K, 11))
    words = [json.loads(r[1])["f0"] for r in rows[2:]]
    assert sorted(words) == list("abcdefghijk")
    out = LdaPredictBatchOp().setPredictionCol("pred").setPredictionDetailCol("d").setSelectedCol("doc") \
        .linkFrom(model, src).collect()
    for r in out:
        p = np.array([float(x) for x in r[2].split(" ")])
        assert abs(p.sum() - 1) < 1e-9 and r[1] == int(np.argmax(p))
    m = Lda().setSelectedCol("doc").setTopicNum(3).setPredictionCol("p").fit(src)
    assert len(m.transform(src).collect()) == 12

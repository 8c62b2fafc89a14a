#!/usr/bin/env python3
"""Host hot-spot sweep: common batch ops on synthetic device tables at production-ish sizes, each run twice (the
first pays one-time costs), the second timed and cProfiled; prints the wall time and the top functions by own
time per op, so Python-level loops over rows / model entries stand out.

    python tools/op_sweep_profile.py [--rows 10000000] [--only kmeans_predict,...]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--only", default="")
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--set", type=int, default=1,
                    help="1: model ops; 2: data processing / SQL / scalers; 3: evaluation / NLP / trees / formats; "
                         "4: IO, more model predicts; 5: SQL joins / sets / order, PCA, normalize, correlation, JSON; "
                         "6: vector mappers, more scalers; 7: more predicts, SQL expressions, regex tokenizer")
    a = ap.parse_args()
    import alink_amd as A
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = A.useLocalEnv(1)
    dev = env.device
    n = a.rows
    g = torch.Generator(device=dev).manual_seed(0)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    # shared tables
    vec = A.RandomVectorSourceBatchOp().setNumRows(n).setSize(128).setNumClusters(100).setClusterStd(1.0) \
        .setCenterScale(4.0).setDtype("bf16").setSeed(7).setOutputCol("vec").getOutputTable()
    F = 20
    cols = [Column(torch.randn(n, generator=g, device=dev, dtype=torch.float64)) for _ in range(F)]
    y = (cols[0].values + 0.5 * cols[1].values > 0).to(torch.int32)
    names = [f"x{i}" for i in range(F)]
    dense = MTable(TableSchema(names + ["label"], [Types.DOUBLE] * F + [Types.INT]), cols + [Column(y)])
    cats = torch.randint(0, 1000, (n,), generator=g, device=dev)
    from alink_amd.common.strings import StringBlock
    vocab = StringBlock.from_list([f"cat_{i}" for i in range(1000)]).to(dev)
    catcol = MTable(TableSchema(["c"], [Types.STRING]), [Column(vocab.take(cats))])
    probs = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    lab = (torch.rand(n, generator=g, device=dev) < probs).to(torch.int32)
    sync()

    km_model = A.KMeansTrainBatchOp().setVectorCol("vec").setK(100).setMaxIter(3) \
        .linkFrom(TableSourceBatchOp(vec))
    lr_model = A.LogisticRegressionTrainBatchOp().setFeatureCols(names).setLabelCol("label").setMaxIter(5) \
        .linkFrom(TableSourceBatchOp(dense))
    si_model = A.StringIndexerTrainBatchOp().setSelectedCol("c").linkFrom(TableSourceBatchOp(catcol))
    oh_model = A.OneHotTrainBatchOp().setSelectedCols(["c"]).linkFrom(TableSourceBatchOp(catcol))
    qd_model = A.QuantileDiscretizerTrainBatchOp().setSelectedCols(names[:5]).setNumBuckets(16) \
        .linkFrom(TableSourceBatchOp(dense))

    det = MTable(TableSchema(["label", "p"], [Types.INT, Types.DOUBLE]), [Column(lab), Column(probs)])

    jobs = {
        "kmeans_predict": lambda: A.KMeansPredictBatchOp().setPredictionCol("pred").setReservedCols([])
        .linkFrom(km_model, TableSourceBatchOp(vec)).getOutputTable().col("pred").values,
        "lr_train": lambda: A.LogisticRegressionTrainBatchOp().setFeatureCols(names).setLabelCol("label")
        .setMaxIter(5).linkFrom(TableSourceBatchOp(dense)).getOutputTable(),
        "lr_predict": lambda: A.LogisticRegressionPredictBatchOp().setPredictionCol("p")
        .setPredictionDetailCol("d").setReservedCols([]).linkFrom(lr_model, TableSourceBatchOp(dense))
        .getOutputTable().col("p").values,
        "string_indexer_train": lambda: A.StringIndexerTrainBatchOp().setSelectedCol("c")
        .linkFrom(TableSourceBatchOp(catcol)).getOutputTable(),
        "string_indexer_predict": lambda: A.StringIndexerPredictBatchOp().setSelectedCol("c").setOutputCol("ci")
        .linkFrom(si_model, TableSourceBatchOp(catcol)).getOutputTable().col("ci").values,
        "onehot_predict": lambda: A.OneHotPredictBatchOp().setSelectedCols(["c"]).setOutputCols(["oh"])
        .linkFrom(oh_model, TableSourceBatchOp(catcol)).getOutputTable().col("oh").values,
        "quantile_predict": lambda: A.QuantileDiscretizerPredictBatchOp().setSelectedCols(names[:5])
        .linkFrom(qd_model, TableSourceBatchOp(dense)).getOutputTable(),
        "vector_assembler": lambda: A.VectorAssemblerBatchOp().setSelectedCols(names).setOutputCol("v")
        .setReservedCols([]).linkFrom(TableSourceBatchOp(dense)).getOutputTable().col("v").values,
        "eval_binary": lambda: A.EvalBinaryClassBatchOp().setLabelCol("label").setPredictionDetailCol("d")
        .linkFrom(A.LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d")
                  .setReservedCols(["label"]).linkFrom(lr_model, TableSourceBatchOp(dense))).collect(),
        "standard_scaler_train": lambda: A.StandardScalerTrainBatchOp().setSelectedCols(names)
        .linkFrom(TableSourceBatchOp(dense)).getOutputTable(),
    }
    if a.set == 2:
        ss = A.StandardScalerTrainBatchOp().setSelectedCols(names).linkFrom(TableSourceBatchOp(dense))
        mm = A.MinMaxScalerTrainBatchOp().setSelectedCols(names).linkFrom(TableSourceBatchOp(dense))
        imp = A.ImputerTrainBatchOp().setSelectedCols(names).setStrategy("MEAN").linkFrom(TableSourceBatchOp(dense))
        src = TableSourceBatchOp(dense)
        catsrc = TableSourceBatchOp(MTable(TableSchema(["c", "x0", "label"], [Types.STRING, Types.DOUBLE, Types.INT]),
                                           [catcol.col("c"), cols[0], Column(y)]))
        jobs = {
            "standard_scaler_predict": lambda: A.StandardScalerPredictBatchOp().linkFrom(ss, src).getOutputTable(),
            "minmax_scaler_predict": lambda: A.MinMaxScalerPredictBatchOp().linkFrom(mm, src).getOutputTable(),
            "imputer_predict": lambda: A.ImputerPredictBatchOp().linkFrom(imp, src).getOutputTable(),
            "feature_hasher": lambda: A.FeatureHasherBatchOp().setSelectedCols(["c", "x0"]).setOutputCol("h")
            .setReservedCols([]).linkFrom(catsrc).getOutputTable().col("h").values,
            "columns_to_vector": lambda: A.ColumnsToVectorBatchOp().setSelectedCols(names).setVectorCol("v")
            .setReservedCols([]).linkFrom(src).getOutputTable().col("v").values,
            "vector_to_columns": lambda: A.VectorToColumnsBatchOp().setSelectedCol("v")
            .setSchemaStr(", ".join(f"y{i} double" for i in range(F))).setReservedCols([])
            .linkFrom(A.VectorAssemblerBatchOp().setSelectedCols(names).setOutputCol("v").setReservedCols([])
                      .linkFrom(src)).getOutputTable(),
            "where": lambda: A.WhereBatchOp().setClause("x0 > 0.5 AND x1 < 0").linkFrom(src).getOutputTable(),
            "select": lambda: A.SelectBatchOp().setClause("x0 + x1 AS s, x2 * 2 AS t, label")
            .linkFrom(src).getOutputTable(),
            "groupby": lambda: A.GroupByBatchOp().setGroupByPredicate("c")
            .setSelectClause("c, COUNT(*) AS n, AVG(x0) AS m").linkFrom(catsrc).getOutputTable(),
            "split": lambda: A.SplitBatchOp().setFraction(0.8).linkFrom(src).getOutputTable(),
            "sample": lambda: A.SampleBatchOp().setRatio(0.1).linkFrom(src).getOutputTable(),
            "numerical_type_cast": lambda: A.NumericalTypeCastBatchOp().setSelectedCols(names[:5])
            .setTargetType("INT").linkFrom(src).getOutputTable(),
            "summarizer": lambda: A.SummarizerBatchOp().setSelectedCols(names).linkFrom(src).collectSummary(),
            "tokenizer": lambda: A.TokenizerBatchOp().setSelectedCol("c").setOutputCol("t")
            .linkFrom(catsrc).getOutputTable(),
        }
    if a.set == 3:
        src = TableSourceBatchOp(dense)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from nlp_count_bench import make_docs
        docsrc = TableSourceBatchOp(MTable(TableSchema(["doc"], [Types.STRING]),
                                           [Column(make_docs(n, 6, 1000, dev))]))
        yreg = cols[0].values * 2 + cols[1].values
        reg = MTable(TableSchema(["label", "p"], [Types.DOUBLE, Types.DOUBLE]),
                     [Column(yreg), Column(yreg + 0.1 * torch.randn(n, generator=g, device=dev, dtype=torch.float64))])
        ml = MTable(TableSchema(["label", "pred"], [Types.INT, Types.INT]),
                    [Column(torch.randint(0, 5, (n,), generator=g, device=dev).to(torch.int32)),
                     Column(torch.randint(0, 5, (n,), generator=g, device=dev).to(torch.int32))])
        small = MTable(TableSchema(names + ["label"], [Types.DOUBLE] * F + [Types.INT]),
                       [Column(c.values[:200000]) for c in cols] + [Column(y[:200000])])
        dt_model = A.DecisionTreeTrainBatchOp().setFeatureCols(names).setLabelCol("label").setMaxDepth(6) \
            .linkFrom(TableSourceBatchOp(small))
        rf_model = A.RandomForestTrainBatchOp().setFeatureCols(names).setLabelCol("label").setMaxDepth(6) \
            .setNumTrees(10).linkFrom(TableSourceBatchOp(small))
        dhc = A.DocHashCountVectorizerTrainBatchOp().setSelectedCol("doc").linkFrom(docsrc)
        dcc = A.DocCountVectorizerTrainBatchOp().setSelectedCol("doc").linkFrom(docsrc)
        jobs = {
            "eval_regression": lambda: A.EvalRegressionBatchOp().setLabelCol("label").setPredictionCol("p")
            .linkFrom(TableSourceBatchOp(reg)).collect(),
            "eval_multiclass": lambda: A.EvalMultiClassBatchOp().setLabelCol("label").setPredictionCol("pred")
            .linkFrom(TableSourceBatchOp(ml)).collect(),
            "binarizer": lambda: A.BinarizerBatchOp().setSelectedCol("x0").setOutputCol("b").setThreshold(0.1)
            .linkFrom(src).getOutputTable(),
            "bucketizer": lambda: A.BucketizerBatchOp().setSelectedCols(["x0", "x1"])
            .setCutsArray([[-1.0, 0.0, 1.0], [0.0]]).linkFrom(src).getOutputTable(),
            "dt_predict": lambda: A.DecisionTreePredictBatchOp().setPredictionCol("p").setReservedCols([])
            .linkFrom(dt_model, src).getOutputTable().col("p").values,
            "rf_predict": lambda: A.RandomForestPredictBatchOp().setPredictionCol("p").setReservedCols([])
            .linkFrom(rf_model, src).getOutputTable().col("p").values,
            "stopwords": lambda: A.StopWordsRemoverBatchOp().setSelectedCol("doc").setOutputCol("o")
            .linkFrom(docsrc).getOutputTable(),
            "ngram": lambda: A.NGramBatchOp().setSelectedCol("doc").setOutputCol("o").linkFrom(docsrc)
            .getOutputTable(),
            "dochash_predict": lambda: A.DocHashCountVectorizerPredictBatchOp().setSelectedCol("doc")
            .setOutputCol("v").linkFrom(dhc, docsrc).getOutputTable().col("v").values,
            "doccount_predict": lambda: A.DocCountVectorizerPredictBatchOp().setSelectedCol("doc")
            .setOutputCol("v").linkFrom(dcc, docsrc).getOutputTable().col("v").values,
            "append_id": lambda: A.AppendIdBatchOp().linkFrom(src).getOutputTable(),
            "columns_to_kv": lambda: A.ColumnsToKvBatchOp().setSelectedCols(names[:5]).setKvCol("kv")
            .setReservedCols([]).linkFrom(src).getOutputTable(),
            "columns_to_json": lambda: A.ColumnsToJsonBatchOp().setSelectedCols(names[:5]).setJsonCol("j")
            .setReservedCols([]).linkFrom(src).getOutputTable(),
        }
    if a.set == 4:
        import tempfile
        src = TableSourceBatchOp(dense)
        tmp = tempfile.mkdtemp()
        csv_path = os.path.join(tmp, "d.csv")
        A.CsvSinkBatchOp().setFilePath(csv_path).setOverwriteSink(True).linkFrom(src)
        schema_str = ", ".join(f"{c} double" for c in names) + ", label int"
        sm = MTable(TableSchema(names + ["label"], [Types.DOUBLE] * F + [Types.INT]),
                    [Column(c.values[:200000]) for c in cols] + [Column(y[:200000])])
        nb_docs = TableSourceBatchOp(MTable(TableSchema(["doc", "label"], [Types.STRING, Types.INT]),
                                            [Column(vocab.take(cats)), Column(y)]))
        sm_src = TableSourceBatchOp(sm)
        softmax_model = A.SoftmaxTrainBatchOp().setFeatureCols(names).setLabelCol("label").setMaxIter(3) \
            .linkFrom(sm_src)
        gmm_model = A.GmmTrainBatchOp().setVectorCol("vec").setK(10).setMaxIter(3) \
            .linkFrom(TableSourceBatchOp(MTable(TableSchema(["vec"], [Types.DENSE_VECTOR]),
                                                [Column(vec.col("vec").values[:200000].float())])))
        nb_model = A.NaiveBayesTextTrainBatchOp().setVectorCol("v").setLabelCol("label") \
            .linkFrom(A.DocHashCountVectorizerPredictBatchOp().setSelectedCol("doc").setOutputCol("v")
                      .linkFrom(A.DocHashCountVectorizerTrainBatchOp().setSelectedCol("doc").setNumFeatures(1000)
                                .linkFrom(nb_docs), nb_docs))
        jobs = {
            "csv_sink": lambda: A.CsvSinkBatchOp().setFilePath(csv_path + ".2").setOverwriteSink(True)
            .linkFrom(src),
            "csv_source": lambda: A.CsvSourceBatchOp().setFilePath(csv_path).setSchemaStr(schema_str)
            .getOutputTable(),
            "collect_rows": lambda: TableSourceBatchOp(sm).collect(),
            "softmax_predict": lambda: A.SoftmaxPredictBatchOp().setPredictionCol("p").setReservedCols([])
            .linkFrom(softmax_model, src).getOutputTable().col("p").values,
            "gmm_predict": lambda: A.GmmPredictBatchOp().setPredictionCol("p").setReservedCols([])
            .linkFrom(gmm_model, TableSourceBatchOp(vec)).getOutputTable().col("p").values,
            "naive_bayes_text_predict": lambda: A.NaiveBayesTextPredictBatchOp().setPredictionCol("p")
            .setReservedCols([]).linkFrom(nb_model, A.DocHashCountVectorizerPredictBatchOp().setSelectedCol("doc")
                                          .setOutputCol("v").linkFrom(
                                              A.DocHashCountVectorizerTrainBatchOp().setSelectedCol("doc")
                                              .setNumFeatures(1000).linkFrom(nb_docs), nb_docs))
            .getOutputTable().col("p").values,
        }
    if a.set == 5:
        src = TableSourceBatchOp(dense)
        keyed = MTable(TableSchema(["k", "x0", "c"], [Types.LONG, Types.DOUBLE, Types.STRING]),
                       [Column(cats.to(torch.int64)), cols[0], Column(vocab.take(cats))])
        dim = MTable(TableSchema(["k2", "name"], [Types.LONG, Types.STRING]),
                     [Column(torch.arange(1000, device=dev)), Column(vocab)])
        ksrc, dsrc = TableSourceBatchOp(keyed), TableSourceBatchOp(dim)
        pca_model = A.PcaTrainBatchOp().setSelectedCols(names).setK(5).linkFrom(src)
        js = A.ColumnsToJsonBatchOp().setSelectedCols(names[:3]).setJsonCol("j").setReservedCols([]) \
            .linkFrom(src).getOutputTable()
        jsrc = TableSourceBatchOp(js)
        vsrc = TableSourceBatchOp(vec)
        jobs = {
            "join": lambda: A.JoinBatchOp().setJoinPredicate("k = k2").setSelectClause("k, x0, name")
            .linkFrom(ksrc, dsrc).getOutputTable(),
            "union_all": lambda: A.UnionAllBatchOp().linkFrom(ksrc, ksrc).getOutputTable(),
            "distinct": lambda: A.DistinctBatchOp().linkFrom(
                TableSourceBatchOp(MTable(TableSchema(["k", "c"], [Types.LONG, Types.STRING]),
                                          [keyed.cols[0], keyed.cols[2]]))).getOutputTable(),
            "order_by": lambda: A.OrderByBatchOp().setClause("x0").setLimit(1000).linkFrom(ksrc).getOutputTable(),
            "pca_predict": lambda: A.PcaPredictBatchOp().setPredictionCol("p").setReservedCols([])
            .linkFrom(pca_model, src).getOutputTable().col("p").values,
            "vector_normalize": lambda: A.VectorNormalizeBatchOp().setSelectedCol("vec").linkFrom(vsrc)
            .getOutputTable().col("vec").values,
            "correlation": lambda: A.CorrelationBatchOp().setSelectedCols(names).linkFrom(src).collect(),
            "json_value": lambda: A.JsonValueBatchOp().setSelectedCol("j").setJsonPath(["$.x0", "$.x1"])
            .setOutputCols(["a", "b"]).linkFrom(jsrc).getOutputTable(),
        }
    if a.set == 6:
        vsrc = TableSourceBatchOp(vec)
        src = TableSourceBatchOp(dense)
        two = MTable(TableSchema(["v1", "v2"], [Types.DENSE_VECTOR, Types.DENSE_VECTOR]),
                     [Column(vec.col("vec").values[:, :8].double()), Column(vec.col("vec").values[:, 8:12].double())])
        mas = A.MaxAbsScalerTrainBatchOp().setSelectedCols(names).linkFrom(src)
        vss = A.VectorStandardScalerTrainBatchOp().setSelectedCol("vec").linkFrom(vsrc)
        jobs = {
            "vector_slice": lambda: A.VectorSliceBatchOp().setSelectedCol("vec").setOutputCol("s")
            .setIndices([0, 3, 5]).setReservedCols([]).linkFrom(vsrc).getOutputTable().col("s").values,
            "vector_elementwise_product": lambda: A.VectorElementwiseProductBatchOp().setSelectedCol("vec")
            .setOutputCol("e").setScalingVector(" ".join(["2.0"] * 128)).setReservedCols([]).linkFrom(vsrc)
            .getOutputTable().col("e").values,
            "vector_interaction": lambda: A.VectorInteractionBatchOp().setSelectedCols(["v1", "v2"])
            .setOutputCol("i").setReservedCols([]).linkFrom(TableSourceBatchOp(two)).getOutputTable()
            .col("i").values,
            "vector_polynomial_expand": lambda: A.VectorPolynomialExpandBatchOp().setSelectedCol("v2")
            .setOutputCol("p").setDegree(2).setReservedCols([]).linkFrom(TableSourceBatchOp(two))
            .getOutputTable().col("p").values,
            "vector_size_hint": lambda: A.VectorSizeHintBatchOp().setSelectedCol("vec").setSize(128)
            .linkFrom(vsrc).getOutputTable(),
            "maxabs_scaler_predict": lambda: A.MaxAbsScalerPredictBatchOp().linkFrom(mas, src).getOutputTable(),
            "vector_standard_scaler_predict": lambda: A.VectorStandardScalerPredictBatchOp().linkFrom(vss, vsrc)
            .getOutputTable().col("vec").values,
        }
    if a.set == 7:
        src = TableSourceBatchOp(dense)
        vsrc = TableSourceBatchOp(vec)
        catsrc = TableSourceBatchOp(MTable(TableSchema(["c", "d"], [Types.STRING, Types.STRING]),
                                           [Column(vocab.take(cats)), Column(vocab.take(cats.flip(0)))]))
        iso = A.IsotonicRegTrainBatchOp().setFeatureCol("x0").setLabelCol("label").linkFrom(src)
        msi = A.MultiStringIndexerTrainBatchOp().setSelectedCols(["c", "d"]).linkFrom(catsrc)
        bkm = A.BisectingKMeansTrainBatchOp().setVectorCol("vec").setK(8).setMaxIter(3).linkFrom(
            TableSourceBatchOp(MTable(vec.schema, [Column(vec.col("vec").values[:100000])])))
        docs = TableSourceBatchOp(MTable(TableSchema(["doc"], [Types.STRING]), [Column(vocab.take(cats))]))
        svocab = StringBlock.from_list([f"w{i % 97} w{i % 89} w{i % 83} w{i % 79} w{i % 7}" for i in range(1000)])
        sents = TableSourceBatchOp(MTable(TableSchema(["doc"], [Types.STRING]), [Column(svocab.to(dev).take(cats))]))
        w2v = A.Word2VecTrainBatchOp().setSelectedCol("doc").setVectorSize(64).setMinCount(1).setNumIter(1) \
            .linkFrom(TableSourceBatchOp(MTable(TableSchema(["doc"], [Types.STRING]), [Column(svocab)])))
        jobs = {
            "isotonic_predict": lambda: A.IsotonicRegPredictBatchOp().setPredictionCol("p").linkFrom(iso, src)
            .getOutputTable().col("p").values,
            "multi_string_indexer_predict": lambda: A.MultiStringIndexerPredictBatchOp().setSelectedCols(["c", "d"])
            .setOutputCols(["ci", "di"]).linkFrom(msi, catsrc).getOutputTable(),
            "kmeans_predict_detail": lambda: A.KMeansPredictBatchOp().setPredictionCol("p")
            .setPredictionDetailCol("d").setReservedCols([]).linkFrom(km_model, vsrc).getOutputTable()
            .col("p").values,
            "bisecting_kmeans_predict": lambda: A.BisectingKMeansPredictBatchOp().setPredictionCol("p")
            .setReservedCols([]).linkFrom(bkm, vsrc).getOutputTable().col("p").values,
            "select_expr": lambda: A.SelectBatchOp().setClause("x0 * 2 + x1 AS a, label").linkFrom(src)
            .getOutputTable(),
            "select_string_fn": lambda: A.SelectBatchOp().setClause("UPPER(c) AS u, CONCAT(c, '_', d) AS cd")
            .linkFrom(catsrc).getOutputTable(),
            "regex_tokenizer": lambda: A.RegexTokenizerBatchOp().setSelectedCol("doc").setPattern("_")
            .linkFrom(docs).getOutputTable(),
            "word2vec_predict": lambda: A.Word2VecPredictBatchOp().setSelectedCol("doc").setOutputCol("v")
            .linkFrom(w2v, sents).getOutputTable().col("v").values,
        }
    only = [s for s in a.only.split(",") if s]
    for name, fn in jobs.items():
        if only and name not in only:
            continue
        try:
            fn()
            sync()
            pr = cProfile.Profile()
            t = time.perf_counter()
            pr.enable()
            fn()
            sync()
            pr.disable()
            wall = time.perf_counter() - t
        except Exception as e:          # keep sweeping; report the op
            print(f"== {name}: FAILED {type(e).__name__}: {e}", flush=True)
            continue
        sio = io.StringIO()
        pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(a.top)
        lines = [ln for ln in sio.getvalue().splitlines() if ln.strip() and ("(" in ln or "ncalls" in ln)]
        print(f"== {name}: {wall:.3f} s for {n} rows ({n / wall:.3g} rows/s)", flush=True)
        for ln in lines[:a.top + 1]:
            print("   " + ln[:170], flush=True)


if __name__ == "__main__":
    main()

"""NLP operators vs the reference docs (docs/en/{tokenizer,regextokenizer,ngram,stopwordsremover,
doccountvectorizer,dochashcountvectorizer}*.md)."""
import json

import pandas as pd
import pytest

from alink_amd import *  # noqa: F401,F403
from alink_amd.models.nlp.text import JiebaSegmenter, java_split

EN = pd.DataFrame({"id": [0, 1, 2], "text": ["That is an English Book!", "Do you like math?", "Have a good day!"]})
ZH = pd.DataFrame({"id": [0, 1, 2, 3, 4], "text": [
    "二手旧书:医学电磁成像", "二手美国文学选读（ 下册 ）李宜燮南开大学出版社 9787310003969",
    "二手正版图解象棋入门/谢恩思主编/华龄出版社", "二手中国糖尿病文献索引", "二手郁达夫文集（ 国内版 ）全十二册馆藏书"]})


def _en():
    return BatchOperator.fromDataframe(EN, schemaStr="id long, text string")


def _zh():
    return BatchOperator.fromDataframe(ZH, schemaStr="id int, text string")


def test_java_split_semantics():
    assert java_split("  a b", r"\s+") == ["", "a", "b"]
    assert java_split("a b  ", r"\s+") == ["a", "b"]
    assert java_split("", " ") == [""]
    assert java_split("a  b", " ") == ["a", "", "b"]


def test_tokenizers_and_ngram_doc():
    assert [r[1] for r in TokenizerBatchOp().setSelectedCol("text").linkFrom(_en()).collect()] == \
        ["that is an english book!", "do you like math?", "have a good day!"]
    out = RegexTokenizerBatchOp().setSelectedCol("text").setGaps(False).setToLowerCase(True) \
        .setOutputCol("token").setPattern("\\w+").linkFrom(_en()).collect()
    assert [r[2] for r in out] == ["that is an english book", "do you like math", "have a good day"]
    assert [r[1] for r in NGramBatchOp().setSelectedCol("text").linkFrom(_en()).collect()] == \
        ["That_is is_an an_English English_Book!", "Do_you you_like like_math?", "Have_a a_good good_day!"]
    box = []
    TokenizerStreamOp().setSelectedCol("text").linkFrom(
        StreamOperator.fromDataframe(EN, schemaStr="id long, text string")).link(CollectStreamOp(box))
    StreamOperator.execute()
    assert sorted(r[1] for r in box) == ["do you like math?", "have a good day!", "that is an english book!"]


def test_segment_stopwords_and_user_dict():
    seg = SegmentBatchOp().setSelectedCol("text").setOutputCol("segment").linkFrom(_zh())
    rem = StopWordsRemoverBatchOp().setSelectedCol("segment").setOutputCol("remover").linkFrom(seg).collect()
    # punctuation is in the default stop list; "二手" starts every document
    assert all(r[3].split(" ")[0] == "二手" for r in rem)
    assert ":" not in rem[0][3] and "/" not in rem[2][3]
    s = JiebaSegmenter(["电磁成像"])
    assert "电磁成像" in s.cut("医学电磁成像")


def test_doc_count_vectorizer_doc_model():
    segt = SegmentBatchOp().setSelectedCol("text").linkFrom(_zh())
    train = DocCountVectorizerTrainBatchOp().setSelectedCol("text").linkFrom(segt)
    rows = train.collect()
    assert rows[0][1] == '{"minTF":"1.0","featureType":"\\"WORD_COUNT\\""}'
    # reference model head (docs/en/doccountvectorizerpredictbatchop.md)
    assert [rows[i][1] for i in range(1, 6)] == [
        '{"f0":"二手","f1":0.0,"f2":0}', '{"f0":"/","f1":1.0986122886681098,"f2":1}',
        '{"f0":"出版社","f1":0.6931471805599453,"f2":2}', '{"f0":"（","f1":0.6931471805599453,"f2":3}',
        '{"f0":"）","f1":0.6931471805599453,"f2":4}']
    pred = DocCountVectorizerPredictBatchOp().setSelectedCol("text").linkFrom(train, segt).collect()
    v = pred[0][1]
    assert v.size() == len(rows) - 1 and v.get(0) == 1.0


def test_doc_hash_count_vectorizer_doc_indices():
    segt = SegmentBatchOp().setSelectedCol("text").linkFrom(_zh())
    train = DocHashCountVectorizerTrainBatchOp().setSelectedCol("text").linkFrom(segt)
    meta = json.loads(train.collect()[0][1])
    assert meta["numFeatures"] == "262144"
    pred = DocHashCountVectorizerPredictBatchOp().setSelectedCol("text").linkFrom(train, segt).collect()
    v1 = pred[1][1]
    # murmur3(word) indices of the reference output: "$262144$0:6.0 37505:1.0 46743:1.0 93228:1.0 ..."
    idx = set(v1.getIndices().tolist())
    assert {0, 37505, 93228} <= idx and v1.get(0) == 6.0
    assert {64444, 206232} <= set(pred[0][1].getIndices().tolist())


def test_word2vec_doc_and_semantics():
    import numpy as np
    from alink_amd.models.nlp.word2vec import huffman
    df = pd.DataFrame({"tokens": ["A B C"]})
    src = BatchOperator.fromDataframe(df, schemaStr="tokens string")
    train = Word2VecTrainBatchOp().setSelectedCol("tokens").setMinCount(1).setVectorSize(4).linkFrom(src)
    rows = train.collect()
    assert sorted(r[0] for r in rows) == ["A", "B", "C"] and rows[0][1].size() == 4
    pred = Word2VecPredictBatchOp().setSelectedCol("tokens").linkFrom(train, src).collect()
    vecs = np.stack([r[1].data for r in rows])
    got = np.array([float(x) for x in pred[0][0].split(" ")])
    np.testing.assert_allclose(got, vecs.mean(0), rtol=1e-12)
    # Huffman: frequent words get short codes, codes are prefix-free
    C, P, L = huffman(np.array([50, 20, 10, 5, 5]))
    assert L[0] <= L[-1] and len({tuple(C[i, :L[i]]) for i in range(5)}) == 5
    # co-occurring words end up closer than unrelated ones
    rng = np.random.default_rng(0)
    docs = [" ".join(rng.permutation(["x1", "x2", "x3"]).tolist()) for _ in range(150)] + \
           [" ".join(rng.permutation(["y1", "y2", "y3"]).tolist()) for _ in range(150)]
    src2 = BatchOperator.fromDataframe(pd.DataFrame({"t": docs}), schemaStr="t string")
    m = Word2VecTrainBatchOp().setSelectedCol("t").setMinCount(1).setVectorSize(8).setNumIter(5) \
        .setWindow(2).linkFrom(src2).collect()
    E = {r[0]: r[1].data / np.linalg.norm(r[1].data) for r in m}
    assert E["x1"] @ E["x2"] > E["x1"] @ E["y1"]


def test_word2vec_batched_hs_learns_on_zipf_topics():
    """The batched CPU skip-gram (models/nlp/word2vec._sgd) on a 10-topic Zipf corpus: HS loss falls clearly
    below ln 2 (its value at the zero-initialised output vectors), and hot ids (the Huffman root is on every
    path) neither stall nor diverge under the bounded duplicate correction."""
    import numpy as np
    import torch
    from alink_amd.models.nlp import word2vec as W
    rng = np.random.default_rng(0)
    V, T = 500, 10
    p = 1.0 / np.arange(1, V // T + 1)
    p /= p.sum()
    docs = [int(rng.integers(T)) * (V // T) + rng.choice(V // T, size=30, p=p) for _ in range(600)]
    cnt = np.bincount(np.concatenate(docs), minlength=V)
    order = np.argsort(-cnt, kind="stable")
    remap = np.empty(V, int)
    remap[order] = np.arange(V)
    docs = [remap[d] for d in docs]
    C, P, L = W.huffman(cnt[order])
    Ct, Pt, Lt = map(torch.as_tensor, (C, P, L))
    inp = torch.rand((V, 32), generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    out = torch.zeros((V - 1, 32), dtype=torch.float64)
    cen, ctx = W._pairs(docs, 5, True, np.random.default_rng(1))
    cen, ctx = torch.as_tensor(cen), torch.as_tensor(ctx)

    def loss():
        nodes, code = Pt[cen], Ct[cen].double()
        mask = torch.arange(C.shape[1])[None, :] < Lt[cen][:, None]
        f = (out[nodes] * inp[ctx][:, None, :]).sum(-1)
        lo = -(torch.nn.functional.logsigmoid(f) * (1 - code) + torch.nn.functional.logsigmoid(-f) * code)
        return float((lo * mask).sum() / mask.sum())
    assert abs(loss() - np.log(2)) < 1e-12
    for _ in range(3):
        W._sgd(inp, out, Ct, Pt, Lt, cen, ctx, 0.025, 4096)
    final = loss()
    assert final < 0.6, final
    assert torch.isfinite(inp).all() and float(inp.abs().max()) < 10


def test_doc_word_split_count_table_function():
    """DocWordSplitCountTest (reference operator/common/nlp): "a b c d a b c" -> (a,2) (b,2) (c,2) (d,1)."""
    from alink_amd.models.nlp.text import DocWordSplitCount
    from alink_amd.operator.batch.source import MemSourceBatchOp
    out = MemSourceBatchOp([("a b c d a b c",)], "f0 string").udtf("f0", ["w", "cnt"], DocWordSplitCount(" "), []) \
        .collect()
    assert [tuple(r) for r in out] == [("a", 2), ("b", 2), ("c", 2), ("d", 1)]


DCV_VOCAB = [("i", 0.6931471805599453, 6), ("e", 0.1823215567939546, 2), ("a", 0.4054651081081644, 0),
             ("b", 0.1823215567939546, 1), ("c", 0.6931471805599453, 7), ("h", 0.4054651081081644, 3),
             ("d", 0.6931471805599453, 4), ("j", 0.6931471805599453, 5), ("g", 0.6931471805599453, 8),
             ("n", 1.0986122886681098, 9), ("f", 1.0986122886681098, 10)]


@pytest.mark.parametrize("ftype,min_tf,text,expect", [
    ("WORD_COUNT", "1.0", "a b c d e a a", "$11$0:3.0 1:1.0 2:1.0 4:1.0 7:1.0"),
    ("TF_IDF", "1.0", "a b c d e", "$11$0:0.08109302162163289 1:0.03646431135879092 2:0.03646431135879092 "
                                   "4:0.13862943611198905 7:0.13862943611198905"),
    ("TF", "1.0", "a b c d e", "$11$0:0.2 1:0.2 2:0.2 4:0.2 7:0.2"),
    ("BINARY", "0.2", "a b c d e a a b e", "$11$0:1.0 1:1.0 2:1.0"),
    ("BINARY", "0.2", "a b c d", "$11$0:1.0 1:1.0 4:1.0 7:1.0")])
def test_doc_count_vectorizer_mapper_reference(ftype, min_tf, text, expect):
    """DocCountVectorizerModelMapperTest: the reference's 11-word model rows; minTF 0.2 keeps words with at least
    20 % of the document's tokens."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import schema_str_to_schema
    from alink_amd.models.nlp.text import DocCountVectorizerModelMapper
    rows = [(0, '{"minTF":"%s","featureType":"\\"%s\\""}' % (min_tf, ftype))] + \
        [((i + 1) * 1048576, '{"f0":"%s","f1":%r,"f2":%d}' % v) for i, v in enumerate(DCV_VOCAB)]
    p = Params().set("selectedCol", "sentence")
    if ftype == "TF":
        p.set("outputCol", "output")
    m = DocCountVectorizerModelMapper(schema_str_to_schema("model_id bigint, model_info string"),
                                      schema_str_to_schema("sentence string"), p)
    m.loadModel(rows)
    assert str(m.map((text,))[-1]) == expect


@pytest.mark.parametrize("ftype,expect", [
    ("TF_IDF", "$20$7:0.0 13:0.06757751801802739 14:-0.25541281188299536 15:-0.047947012075296815"),
    ("WORD_COUNT", "$20$7:1.0 13:1.0 14:3.0 15:1.0"),
    ("TF", "$20$7:0.16666666666666666 13:0.16666666666666666 14:0.5 15:0.16666666666666666"),
    ("BINARY", "$20$7:1.0 13:1.0 14:1.0 15:1.0"),
    ("IDF", "$20$7:0.0 13:0.4054651081081644 14:-0.5108256237659907 15:-0.2876820724517809")])
def test_doc_hash_count_vectorizer_mapper_reference(ftype, expect):
    """DocHashCountVectorizerModelMapperTest: 20 hash buckets, the reference's IDF row, text "a b c d a a "."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import schema_str_to_schema
    from alink_amd.models.nlp.text import DocHashCountVectorizerModelMapper
    rows = [(0, '{"numFeatures":"20","minTF":"1.0","featureType":"\\"%s\\""}' % ftype),
            (1048576, '{"16":0.4054651081081644,"7":0.0,"13":0.4054651081081644,"14":-0.5108256237659907,'
                      '"15":-0.2876820724517809}')]
    m = DocHashCountVectorizerModelMapper(schema_str_to_schema("model_id bigint, model_info string"),
                                          schema_str_to_schema("sentence string"), Params().set("selectedCol", "sentence"))
    m.loadModel(rows)
    assert str(m.map(("a b c d a a ",))[0]) == expect


def _siso(cls, **params):
    from alink_amd.common.params import Params
    from alink_amd.common.types import schema_str_to_schema
    p = Params().set("selectedCol", "sentence")
    for k, v in params.items():
        p.set(k, v)
    return cls(schema_str_to_schema("sentence string"), p)


def test_stop_words_remover_mapper_reference():
    """StopWordsRemoverMapperTest: the bundled English / Chinese stop words plus "Test", case-insensitive by
    default, case-sensitive on request."""
    from alink_amd.models.nlp.text import StopWordsRemoverMapper
    m = _siso(StopWordsRemoverMapper, stopWords=["Test"])
    assert m.map(("This is a unit test for filtering stopWords",))[0] == "unit filtering stopWords"
    assert m.map(("Filter stopWords test",))[0] == "Filter stopWords"
    assert m.map(("这 是 停用词 过滤 的 单元 测试",))[0] == "停用词 过滤 单元 测试"
    m = _siso(StopWordsRemoverMapper, caseSensitive=True, stopWords=["Test"])
    assert m.map(("This is a unit test for filtering stopWords",))[0] == "This unit test filtering stopWords"
    assert m.map(("Filter stopWords test",))[0] == "Filter stopWords test"


@pytest.mark.parametrize("n,expect", [(None, "This_is is_a a_unit unit_test test_for for_mapper"),
                                      (3, "This_is_a is_a_unit a_unit_test unit_test_for test_for_mapper"),
                                      (10, "")])
def test_ngram_mapper_reference(n, expect):
    """NGramMapperTest."""
    from alink_amd.models.nlp.text import NGramMapper
    m = _siso(NGramMapper, **({} if n is None else {"n": n}))
    assert m.map(("This is a unit test for mapper",))[0] == expect


def test_doc_hash_count_vectorizer_tensor_counts_equal_per_document_counter():
    """The tensor trainer (device split + murmur3 + bincount + one int64 all-reduce) writes exactly the model of the
    per-document form it replaced: Java split semantics (leading / doubled / trailing spaces, empty and NULL
    documents), non-ASCII words, fractional minDF."""
    import math
    import random
    from collections import Counter
    from alink_amd.common.javafmt import gson_dumps
    from alink_amd.models.feature.encoders import murmur3_index
    from alink_amd.models.nlp.text import java_split
    random.seed(3)
    docs = ["", " ", "a b", " a  b ", "héllo wörld  x", None, "   ", "中文 分词 中文"]
    for _ in range(400):
        docs.append(" ".join(random.choice(["a", "b", "", "c", "dé", "ß", "w%d" % random.randint(0, 50)])
                             for _ in range(random.randint(0, 9))) if random.random() > 0.05 else None)
    src = BatchOperator.fromDataframe(pd.DataFrame({"t": docs}), schemaStr="t string")
    for nf, min_df in ((32, 1.0), (1 << 10, 3.0), (1 << 10, 0.01)):
        got = DocHashCountVectorizerTrainBatchOp().setSelectedCol("t").setNumFeatures(nf).setMinDF(min_df) \
            .linkFrom(src).collect()
        cnt = Counter()
        for v in docs:
            words = java_split(str(v), " ") if v is not None else []
            if words:
                cnt.update(murmur3_index(words, nf).tolist())
        md = min_df if min_df >= 1.0 else min_df * len(docs)
        idf = {int(k): math.log((len(docs) + 1.0) / (c + 1.0)) for k, c in cnt.items() if c >= md}
        # HashMap<Integer, Double> iteration (keys < capacity): ascending k ^ (k >>> 16)
        want = "{" + ",".join('"%d":%s' % (k, gson_dumps(idf[k])) for k in sorted(idf, key=lambda k: k ^ (k >> 16))) \
            + "}"
        data = [r[1] for r in got if r[0] != 0 and r[1] is not None]
        assert data == [want]


def _random_docs(n, seed):
    import random
    random.seed(seed)
    docs = ["", " ", "a b", " a  b ", "héllo wörld  x", None, "   ", "中文 分词 中文"]
    for _ in range(n):
        docs.append(" ".join(random.choice(["a", "b", "", "c", "dé", "ß", "w%d" % random.randint(0, 50)])
                             for _ in range(random.randint(0, 9))) if random.random() > 0.05 else None)
    return docs


def test_doc_count_vectorizer_tensor_stats_equal_counter_path(monkeypatch):
    """DocCountVectorizer's tensor word statistics (device split, exact dictionary encoding, bincounts) train the
    same model as the per-document Counter path, which stays as the fallback of a hash collision."""
    from alink_amd.ops import strings as S
    docs = _random_docs(500, 5)
    src = BatchOperator.fromDataframe(pd.DataFrame({"t": docs}), schemaStr="t string")

    def train():
        return DocCountVectorizerTrainBatchOp().setSelectedCol("t").setMinDF(2.0).setFeatureType("TF_IDF") \
            .linkFrom(src).collect()
    a = train()
    monkeypatch.setattr(S, "unique_ids", lambda blk: None)
    b = train()
    assert a == b and len(a) > 10


def test_split_tokens_and_unique_ids_host():
    """ops/strings.split_tokens == java_split per document; unique_ids is an exact dictionary encoding."""
    from alink_amd.common.strings import StringBlock
    from alink_amd.ops.strings import split_tokens, unique_ids
    docs = _random_docs(300, 9)
    tok, doc = split_tokens(StringBlock.from_list(docs))
    got = {}
    for t, d in zip(tok.to_list(), doc.tolist()):
        got.setdefault(d, []).append(t)
    for i, s in enumerate(docs):
        assert got.get(i, []) == ([] if s is None else java_split(s, " "))
    ids, rep = unique_ids(tok)
    toks = tok.to_list()
    first = {}
    for i, t in enumerate(toks):
        first.setdefault(t, i)
    assert sorted(first.values()) == sorted(rep.tolist())
    for i, t in enumerate(toks):
        assert toks[int(rep[ids[i]])] == t


def test_doc_count_model_rows_fast_format_equals_gson():
    """The DocCountVectorizer model strings from the C++ double formatter equal the generic Gson serializer's,
    escaped words, long vocabularies and Java double edge values included."""
    import math
    from alink_amd.common.javafmt import gson_dumps
    from alink_amd.models.nlp.text import _Tuple3, _tuple3_rows
    words = [f"w{i}" for i in range(300)] + ['q"uote', "back\\slash", "tab\there", "é", "", " x"]
    keep = [(w, 1, v) for w, v in zip(words, [math.log((1.0 + 1e7) / (1.0 + i)) for i in range(len(words))])]
    keep += [("a", 1, 0.0), ("b", 1, 1e-3), ("c", 1, 1e7), ("d", 1, 123456789.125), ("e", 1, 5e-324)]
    ref = [gson_dumps(_Tuple3(w, float(idf), i), java_map_order=False) for i, (w, _, idf) in enumerate(keep)]
    assert _tuple3_rows(keep) == ref
    assert _tuple3_rows([]) == []


def test_tokenizer_packed_block_equals_row_path():
    """Tokenizer on a packed block (byte-parallel lower case + whitespace runs) equals the per-row mapper: leading /
    trailing / mixed whitespace runs, all-whitespace and empty strings, nulls; non-ASCII text takes the row path."""
    from alink_amd.common.params import Params
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.nlp.text import TokenizerMapper
    vals = ["Hello  World", "  Lead and TRAIL \\t\\n", "", "   ", None, "a\\tb\\x0bc\\x0cd\\re", "MiXeD 123 !@#",
            "x", " y", "z ", "A  B   C    D"] * 3
    for extra in ([], ["Ünïcode Tëxt"]):
        v = vals + extra
        mt = MTable(TableSchema(["s"], [Types.STRING]), [Column(StringBlock.from_list(v))])
        m = TokenizerMapper(mt.schema, Params().set("selectedCol", "s").set("outputCol", "t"))
        got = m._map_columns(mt)[0].to_list()
        assert got == [m.mapColumn(x) for x in v]


@pytest.mark.parametrize("ftype", ["WORD_COUNT", "TF_IDF", "TF", "BINARY", "IDF"])
@pytest.mark.parametrize("min_tf", [1.0, 2.0, 0.3])
def test_doc_vectorizer_predict_packed_equals_row_path(ftype, min_tf):
    """DocCount / DocHashCount predict on a packed document column (token arrays on the device) equal the per-row
    mapper: repeated words, double spaces (empty tokens), unseen words, nulls, every feature type, absolute and
    relative minTF."""
    from alink_amd.common.params import Params
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.nlp import text as T
    train = ["a b c a", "b b d", "c a e", "e e e b", "f"] * 4
    docs = ["a b c a a", "b  b d", None, "zz a", "e", "", "a a a b b c d e f"] * 3
    mtr = MTable(TableSchema(["doc"], [Types.STRING]), [Column(list(train))])
    for kind in ("count", "hash"):
        p = Params().set("selectedCol", "doc").set("minTF", min_tf).set("featureType", ftype)
        if kind == "count":
            rows = T.train_doc_count_vectorizer(mtr, p)
            mapper_cls = T.DocCountVectorizerModelMapper
        else:
            rows = T.train_doc_hash_count_vectorizer(mtr, p.clone().set("numFeatures", 64))
            mapper_cls = T.DocHashCountVectorizerModelMapper
        mt = MTable(TableSchema(["doc"], [Types.STRING]), [Column(StringBlock.from_list(docs))])
        m = mapper_cls(None, mt.schema, Params().set("selectedCol", "doc").set("outputCol", "v"))
        m.loadModel(rows)
        got = m._map_columns(mt)[0].to_list()
        ref = [m._map_row_values([d])[0] for d in docs]
        assert [str(x) for x in got] == [str(x) for x in ref], kind


@pytest.mark.parametrize("n", [2, 3])
def test_stopwords_and_ngram_packed_equal_row_path(n):
    """StopWordsRemover and NGram on packed documents (device split + byte-parallel rebuild) equal the row
    mappers: double spaces (empty tokens), leading / trailing spaces, case, documents shorter than n, nulls."""
    from alink_amd.common.params import Params
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.nlp.text import NGramMapper, StopWordsRemoverMapper
    docs = ["the quick brown fox", "A  The an apple", " leading and", "trailing the ", "", None, "one",
            "x y", "THE The the", "a b c d e f g", "  ", "é à ü", "日本 語 テキスト"] * 3
    mt = MTable(TableSchema(["d"], [Types.STRING]), [Column(StringBlock.from_list(docs))])
    for case in (False, True):
        m = StopWordsRemoverMapper(mt.schema, Params().set("selectedCol", "d").set("outputCol", "o")
                                   .set("caseSensitive", case))
        assert m._map_columns(mt)[0].to_list() == [m.mapColumn(x) for x in docs]
    g = NGramMapper(mt.schema, Params().set("selectedCol", "d").set("outputCol", "o").set("n", n))
    assert g._map_columns(mt)[0].to_list() == [g.mapColumn(x) for x in docs]


def test_has_strip_space_matches_python_strip():
    """has_strip_space flags exactly the texts in which Python's strip() could remove more than spaces."""
    import torch
    from alink_amd.ops.strings import has_strip_space
    for ch in ["\t", "\n", "\x0b", "\x0c", "\r", "\x1c", "\x1f", "\x85", "\xa0", "\u1680", "\u2000", "\u200a",
               "\u2028", "\u2029", "\u202f", "\u205f", "\u3000"]:
        assert ch.strip() == ""
        assert has_strip_space(torch.frombuffer(bytearray(("a" + ch + "b").encode()), dtype=torch.uint8))
    for txt in ["plain text", "é à ü", "日本語", "\u200b zero width", "\u180e"]:
        assert has_strip_space(torch.frombuffer(bytearray(txt.encode()), dtype=torch.uint8)) is False


@pytest.mark.parametrize("pattern,lower,min_len", [("_", True, 1), ("\\|", False, 2), (",", True, 0),
                                                   ("\\s+", True, 1)])
def test_regex_tokenizer_literal_delimiter_columnar(pattern, lower, min_len):
    """RegexTokenizer on a one-character delimiter runs on packed bytes and equals the regex row path (leading
    empties kept, trailing dropped, minimum length, ASCII lower-casing, nulls); other patterns use the row path."""
    from alink_amd.common.params import Params
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.nlp.text import RegexTokenizerMapper
    docs = ["Ab_cD_e", "_x__Y_", "", None, "a|B||c|", "no delim", ",,a,b,,", "Q_r,s|T"]
    schema = TableSchema(["s"], [Types.STRING])
    mt = MTable(schema, [Column(StringBlock.from_list(docs))])
    m = RegexTokenizerMapper(schema, Params().set("selectedCol", "s").set("pattern", pattern)
                             .set("toLowerCase", lower).set("minTokenLength", min_len))
    fast = m._map_columns(mt)[0].to_list()
    slow = [m.mapColumn(d) for d in docs]
    assert fast == slow


@pytest.mark.parametrize("method", ["AVG", "SUM", "MIN", "MAX"])
def test_word2vec_predict_columnar(method):
    """Word2Vec document vectors over packed documents (position-by-position fold) equal the per-document row
    path bit for bit: unknown words, repeats, empty and null documents, all-unknown documents."""
    import numpy as np
    from alink_amd.common.params import Params
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.nlp.word2vec import Word2VecModelMapper
    rng = np.random.default_rng(0)
    vocab = ["a", "bb", "c", "dé"]
    schema = TableSchema(["s"], [Types.STRING])
    m = Word2VecModelMapper(TableSchema(["word", "vec"], [Types.STRING, Types.STRING]), schema,
                            Params().set("selectedCol", "s").set("outputCol", "o").set("predMethod", method))
    m.embed = {w: rng.standard_normal(5) for w in vocab}
    docs = ["a bb c", "zz a a", "", None, "q r", "dé  c bb a bb", " a", "c"] * 3
    mt = MTable(schema, [Column(StringBlock.from_list(docs))])
    fast = m._map_columns(mt)[0]
    assert isinstance(fast.values, StringBlock)
    slow = [m._map_row_values((d,))[0] for d in docs]
    assert fast.to_list() == slow

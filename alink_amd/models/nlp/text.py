"""Text processing: tokenizers, stop-word removal, n-grams, Chinese segmentation and document vectorizers.

Reference: ``A/operator/common/nlp/{TokenizerMapper,RegexTokenizerMapper,StopWordsRemoverMapper,NGramMapper,
SegmentMapper,DocCountVectorizerModelMapper,DocHashCountVectorizerModelMapper,FeatureType}.java``,
``A/operator/batch/nlp/{DocCountVectorizerTrainBatchOp,DocHashCountVectorizerTrainBatchOp}.java`` and the
Jieba segmenter (``jiebasegment/``; HMM constants of ``viterbi/FinalSeg``, emissions from the bundled
``prob_emit.txt``).  Tokens are joined by a single space (``NLPConstant.WORD_DELIMITER``); Java's
``String.split`` / ASCII ``\\w``/``\\s`` regex semantics are reproduced.

The vectorizers' train side is a global word / hashed-index count (local ``Counter`` per rank merged with one
object all-gather); prediction emits ``SparseVector``s in the reference's value conventions
(TF, TF_IDF, IDF, BINARY, WORD_COUNT).
"""
from __future__ import annotations

import math
import os
import re
from collections import Counter
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ...common.javafmt import _gson_escape, gson_dumps
from ...common.linalg import SparseVector
from ...common.mapper import SISOMapper, ModelMapper, OutputColsHelper, find_col_index
from ...common.model.converter import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...parallel import comm

__all__ = ["java_split", "DocWordSplitCount", "TokenizerMapper", "RegexTokenizerMapper", "StopWordsRemoverMapper", "NGramMapper",
           "SegmentMapper", "JiebaSegmenter", "DocCountVectorizerModelMapper", "DocHashCountVectorizerModelMapper",
           "train_doc_count_vectorizer", "train_doc_hash_count_vectorizer", "FEATURE_TYPES", "WORD_DELIMITER"]

WORD_DELIMITER = " "
_RES = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "resources")


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


def java_split(s: str, pattern: str) -> List[str]:
    """``String.split(regex)``: trailing empty strings dropped; a leading empty string only for a
    positive-width match at index 0; the empty input gives ``[""]``."""
    if s == "":
        return [""]
    if pattern == " ":
        parts = s.split(" ")
    else:
        parts = re.split(pattern, s, flags=re.ASCII)
        if parts and parts[0] == "":
            m = re.match(pattern, s, flags=re.ASCII)
            if m is not None and m.end() == 0:
                parts = parts[1:]
    while parts and parts[-1] == "":
        parts.pop()
    return parts


class TokenizerMapper(SISOMapper):
    """Lower-case, split on ``\\s+``."""

    def mapColumn(self, v):
        if v is None:
            return None
        return " ".join(java_split(str(v).lower(), r"\s+")).strip()

    def _map_columns(self, mt):
        """A packed string column is tokenized byte-parallel where it lives (``ops/strings.tokenize_ws_lower``);
        anything else (or non-ASCII text) row by row."""
        from ...common.strings import StringBlock
        from ...ops.strings import tokenize_ws_lower
        col = mt.col(self.selected)
        if isinstance(col.values, StringBlock) and col.nulls is None:
            blk = tokenize_ws_lower(col.values)
            if blk is not None:
                return [Column(blk)]
        return super()._map_columns(mt)


class RegexTokenizerMapper(SISOMapper):
    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        p = self.params
        self.pattern = _pget(p, "pattern", r"\s+")
        self.gaps = bool(_pget(p, "gaps", True))
        self.min_len = int(_pget(p, "minTokenLength", 1))
        self.lower = bool(_pget(p, "toLowerCase", True))
        self._re = re.compile(self.pattern, flags=re.ASCII)

    def mapColumn(self, v):
        if v is None:
            return None
        s = str(v).lower() if self.lower else str(v)
        toks = java_split(s, self.pattern) if self.gaps else [m.group() for m in self._re.finditer(s)]
        return WORD_DELIMITER.join(t for t in toks if len(t) >= self.min_len)

    def _literal_byte(self):
        """The delimiter byte when ``pattern`` (gaps mode) matches exactly one fixed ASCII character."""
        pat = self.pattern
        if len(pat) == 2 and pat[0] == "\\" and not pat[1].isalnum() and pat[1].isascii():
            pat = pat[1]
        if len(pat) == 1 and pat.isascii() and pat not in ".^$*+?{}[]|()\\" and ord(pat) >= 0x20:
            return ord(pat)
        return None

    def _map_columns(self, mt):
        """A one-character delimiter over packed documents: lower-casing (ASCII bytes), Java split and the
        minimum-length filter on the device, tokens joined back byte-parallel -- the row path's text."""
        from ...common.strings import StringBlock
        from ...ops.strings import join_tokens, split_tokens
        col = mt.col(self.selected)
        blk = col.values
        d = self._literal_byte() if self.gaps else None
        if d is None or not isinstance(blk, StringBlock) or col.nulls is not None or not len(blk) or \
                (blk.data.numel() and bool((blk.data >= 0x80).any())):
            return super()._map_columns(mt)
        if self.lower:
            up = (blk.data >= 0x41) & (blk.data <= 0x5A)
            blk = StringBlock(torch.where(up, blk.data + 32, blk.data), blk.offsets, blk.nulls)
        tok, doc = split_tokens(blk, d)
        toff = tok.offsets.to(doc.device)
        keep = (toff[1:] - toff[:-1]) >= self.min_len
        return [Column(join_tokens(tok, doc, keep, len(blk), blk.nulls))]


_STOP_CACHE: Optional[List[str]] = None


def default_stop_words() -> List[str]:
    global _STOP_CACHE
    if _STOP_CACHE is None:
        with open(os.path.join(_RES, "stop.txt"), encoding="utf-8") as f:
            _STOP_CACHE = [ln.rstrip("\n").rstrip("\r") for ln in f if ln.rstrip("\n").rstrip("\r")]
    return _STOP_CACHE


class StopWordsRemoverMapper(SISOMapper):
    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.case = bool(_pget(self.params, "caseSensitive", False))
        words = list(_pget(self.params, "stopWords", []) or []) + default_stop_words()
        self.stop = {w if self.case else w.lower() for w in words}

    def mapColumn(self, v):
        if v is None:
            return None
        out = [t for t in java_split(str(v), WORD_DELIMITER)
               if t and (t if self.case else t.lower()) not in self.stop]
        return WORD_DELIMITER.join(out)

    def _map_columns(self, mt):
        """Packed documents: split on the device, one stop-word test per DISTINCT token, the kept tokens joined
        back byte-parallel (``ops/strings.join_tokens``)."""
        from ...common.strings import StringBlock
        from ...ops.strings import join_tokens, split_tokens, unique_ids
        col = mt.col(self.selected)
        blk = col.values
        if isinstance(blk, StringBlock) and col.nulls is None and len(blk):
            tok, doc = split_tokens(blk)
            enc = unique_ids(tok)
            if enc is not None:
                ids, rep = enc
                words = tok.take(rep).to_list()
                ok = torch.tensor([bool(w) and (w if self.case else w.lower()) not in self.stop for w in words]
                                  or [False], dtype=torch.bool)
                keep = ok.to(ids.device)[ids] if len(words) else torch.zeros(0, dtype=torch.bool,
                                                                             device=ids.device)
                return [Column(join_tokens(tok, doc, keep, len(blk), blk.nulls))]
        return super()._map_columns(mt)


class NGramMapper(SISOMapper):
    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.n = int(_pget(self.params, "n", 2))
        if self.n <= 0:
            raise ValueError("N must be positive!")

    def mapColumn(self, v):
        if v is None:
            return None
        toks = java_split(str(v), WORD_DELIMITER)
        grams = ["_".join(toks[i:i + self.n]) for i in range(0, 1 + len(toks) - self.n)]
        return WORD_DELIMITER.join(grams).strip()

    def _map_columns(self, mt):
        """Packed documents with n >= 2: split on the device and the grams assembled byte-parallel
        (``ops/strings.ngram_join``); text holding a character strip() removes (other than the space, which never
        ends a gram) row by row."""
        from ...common.strings import StringBlock
        from ...ops.strings import has_strip_space, ngram_join, split_tokens
        col = mt.col(self.selected)
        blk = col.values
        if isinstance(blk, StringBlock) and col.nulls is None and len(blk) and self.n >= 2:
            if not has_strip_space(blk.data):
                tok, doc = split_tokens(blk)
                return [Column(ngram_join(tok, doc, len(blk), self.n, blk.nulls))]
        return super()._map_columns(mt)


# ---------------------------------------------------------------------------------------------------
# Jieba-style segmentation: prefix-dictionary DAG + max-probability route + HMM (BMES Viterbi) for OOV runs
# ---------------------------------------------------------------------------------------------------
_START = {"B": -0.26268660809250016, "E": -3.14e100, "M": -3.14e100, "S": -1.4652633398537678}
_TRANS = {"B": {"E": -0.510825623765990, "M": -0.916290731874155},
          "E": {"B": -0.5897149736854513, "S": -0.8085250474669937},
          "M": {"E": -0.33344856811948514, "M": -1.2603623820268226},
          "S": {"B": -0.7211965654669841, "S": -0.6658631448798212}}
_PREV = {"B": "ES", "M": "MB", "S": "SE", "E": "BM"}
_MIN = -3.14e100
_EMIT: Optional[Dict[str, Dict[str, float]]] = None


def _emit():
    global _EMIT
    if _EMIT is None:
        em: Dict[str, Dict[str, float]] = {}
        cur = None
        with open(os.path.join(_RES, "prob_emit.txt"), encoding="utf-8") as f:
            for line in f:
                line = line.rstrip("\n").rstrip("\r")
                if not line:
                    continue
                parts = line.split("\t")
                if len(parts) == 1:
                    cur = em.setdefault(parts[0][0], {})
                else:
                    cur[parts[0][0]] = float(parts[1])
        _EMIT = em
    return _EMIT


_RE_HAN = re.compile(r"([一-鿕a-zA-Z0-9+#&\._%\-]+)")
_RE_SKIP = re.compile(r"(\r\n|\s)")
_RE_CHINESE = re.compile(r"[一-鿕]")
_RE_OTHER = re.compile(r"[a-zA-Z0-9]+(?:\.\d+)?%?")


def _viterbi(s: str) -> List[str]:
    em = _emit()
    V = [{st: _START[st] + em.get(st, {}).get(s[0], _MIN) for st in "BMES"}]
    path = {st: st for st in "BMES"}
    for i in range(1, len(s)):
        V.append({})
        newpath = {}
        for y in "BMES":
            ep = em.get(y, {}).get(s[i], _MIN)
            best, bk = None, None
            for y0 in _PREV[y]:
                p = V[i - 1][y0] + _TRANS[y0].get(y, _MIN) + ep
                if best is None or best <= p:
                    best, bk = p, y0
            V[i][y] = best
            newpath[y] = path[bk] + y
        path = newpath
    last = path["S"] if V[-1]["E"] < V[-1]["S"] else path["E"]
    out, begin, nxt = [], 0, 0
    for i, pos in enumerate(last):
        if pos == "B":
            begin = i
        elif pos == "E":
            out.append(s[begin:i + 1])
            nxt = i + 1
        elif pos == "S":
            out.append(s[i])
            nxt = i + 1
    if nxt < len(s):
        out.append(s[nxt:])
    return out


def _hmm_cut(s: str) -> List[str]:
    out, buf_c, buf_o = [], [], []

    def flush_other():
        if buf_o:
            text = "".join(buf_o)
            pos = 0
            for m in _RE_OTHER.finditer(text):
                if m.start() > pos:
                    out.extend(list(text[pos:m.start()]))
                out.append(m.group())
                pos = m.end()
            if pos < len(text):
                out.extend(list(text[pos:]))
            buf_o.clear()

    for ch in s:
        if _RE_CHINESE.match(ch):
            flush_other()
            buf_c.append(ch)
        else:
            if buf_c:
                out.extend(_viterbi("".join(buf_c)))
                buf_c.clear()
            buf_o.append(ch)
    if buf_c:
        out.extend(_viterbi("".join(buf_c)))
    flush_other()
    return out


class JiebaSegmenter:
    """Dictionary DAG + HMM segmenter.  The main Jieba dictionary (``dict.txt``) is not part of the reference
    snapshot either; when ``alink_amd/resources/dict.txt`` is absent the DAG uses only user words and every
    out-of-vocabulary run goes through the HMM (parity unpinned)."""

    def __init__(self, user_words: Sequence[str] = ()):
        self.freq: Dict[str, int] = {}
        path = os.path.join(_RES, "dict.txt")
        if os.path.exists(path):
            with open(path, encoding="utf-8") as f:
                for line in f:
                    parts = line.strip().split(" ")
                    if len(parts) >= 2:
                        self.freq[parts[0]] = int(parts[1])
        self.total = max(1, sum(self.freq.values()))
        for w in user_words:
            self.add_word(w)

    def add_word(self, w: str, freq: int = 3):
        w = w.strip()
        if not w:
            return
        self.freq[w] = freq
        self.total += freq
        for i in range(1, len(w)):
            self.freq.setdefault(w[:i], 0)

    def _dag(self, s):
        dag = {}
        n = len(s)
        for k in range(n):
            ends = []
            i = k
            frag = s[k]
            while i < n and frag in self.freq:
                if self.freq[frag]:
                    ends.append(i)
                i += 1
                frag = s[k:i + 1]
            dag[k] = ends or [k]
        return dag

    def _cut_block(self, s):
        dag = self._dag(s)
        n = len(s)
        logt = math.log(self.total)
        route = {n: (0.0, 0)}
        for i in range(n - 1, -1, -1):
            route[i] = max((math.log(self.freq.get(s[i:x + 1]) or 1) - logt + route[x + 1][0], x) for x in dag[i])
        out, buf, x = [], "", 0
        while x < n:
            y = route[x][1] + 1
            w = s[x:y]
            if y - x == 1:
                buf += w
            else:
                if buf:
                    out.extend(self._flush(buf))
                    buf = ""
                out.append(w)
            x = y
        if buf:
            out.extend(self._flush(buf))
        return out

    def _flush(self, buf):
        if len(buf) == 1:
            return [buf]
        if not self.freq.get(buf):
            return _hmm_cut(buf)
        return list(buf)

    def cut(self, text: str, search: bool = True) -> List[str]:
        out = []
        for blk in _RE_HAN.split(text):
            if not blk:
                continue
            if _RE_HAN.fullmatch(blk):
                for w in self._cut_block(blk):
                    if search:
                        for k in (2, 3):
                            if len(w) > k:
                                out.extend(w[i:i + k] for i in range(len(w) - k + 1) if self.freq.get(w[i:i + k]))
                    out.append(w)
            else:
                out.extend(t for t in _RE_SKIP.split(blk) if t)   # whitespace stays a token, as in Jieba
        return out


class SegmentMapper(SISOMapper):
    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.seg = JiebaSegmenter(_pget(self.params, "userDefinedDict", []) or [])

    def mapColumn(self, v):
        if v is None:
            return None
        return WORD_DELIMITER.join(self.seg.cut(str(v))).strip()


# ---------------------------------------------------------------------------------------------------
# document vectorizers
# ---------------------------------------------------------------------------------------------------
FEATURE_TYPES = {
    "IDF": lambda idf, tf, ratio: idf,
    "WORD_COUNT": lambda idf, tf, ratio: tf,
    "TF_IDF": lambda idf, tf, ratio: idf * tf * ratio,
    "BINARY": lambda idf, tf, ratio: 1.0,
    "TF": lambda idf, tf, ratio: tf * ratio,
}


def _ename(v, default):
    return default if v is None else str(getattr(v, "name", v)).upper()


class DocWordSplitCount:
    """Table function doc -> (word, count) rows, words in first-occurrence order (reference
    ``A/operator/common/nlp/DocWordSplitCount.java``); usable with ``BatchOperator.udtf``."""

    result_types = ["STRING", "LONG"]

    def __init__(self, delimiter: str = " "):
        self.delimiter = delimiter

    def __call__(self, doc):
        if doc is None:
            return []
        counts = Counter(w for w in java_split(str(doc), self.delimiter) if w)
        return [(w, int(c)) for w, c in counts.items()]


class _Tuple3:
    __gson_fields__ = ("f0", "f1", "f2")

    def __init__(self, a, b, c):
        self.f0, self.f1, self.f2 = a, b, c


def _doc_word_stats(mt: MTable, col: str):
    """(words, word count int64, document frequency int64) of this rank's documents, built as tensors: the device
    split (``ops/strings.split_tokens``), an exact dictionary encoding of the non-empty tokens (``unique_ids``),
    ``bincount`` of the word ids for the counts and of the distinct (document, word) pairs for the document
    frequency.  Only the distinct words become Python strings.  None when the encoding meets a hash collision."""
    from ...ops.strings import split_tokens, unique_ids
    from ..feature.encoders import feature_device
    dev = feature_device()
    tok, doc = split_tokens(_string_block(mt, col, dev))
    ne = tok.lengths() > 0
    tok, doc = tok.take(torch.nonzero(ne).reshape(-1)), doc[ne]
    enc = unique_ids(tok)
    if enc is None:
        return None
    ids, rep = enc
    u = int(rep.numel())
    wc = torch.bincount(ids, minlength=u)
    pair = torch.unique(doc * max(u, 1) + ids)
    dfv = torch.bincount(pair % max(u, 1), minlength=u)
    words = tok.take(rep).to_list()
    return words, wc.cpu().numpy(), dfv.cpu().numpy()


def train_doc_count_vectorizer(mt: MTable, params: Params) -> List[tuple]:
    """Vocabulary by total word count (ties: ascending word), document-frequency filter, idf
    ``log((1 + N) / (1 + df))`` (``DocCountVectorizerTrainBatchOp.CalcIdf``)."""
    col = params.get("selectedCol")
    ndoc = mt.num_rows    # COUNT(1) counts null documents too
    stats = _doc_word_stats(mt, col)
    if stats is not None:
        words, wc, dfv = stats
        wc_c = dict(zip(words, wc.tolist()))
        df_c = dict(zip(words, dfv.tolist()))
    else:
        df_c, wc_c = Counter(), Counter()
        for v in mt.column_values(col):
            if v is None or str(v) == "":
                continue
            cnt = Counter(w for w in java_split(str(v), WORD_DELIMITER) if w)
            for w, c in cnt.items():
                df_c[w] += 1
                wc_c[w] += c
    docs = int(sum(comm.all_gather_object(ndoc))) if comm.get_world_size() > 1 else ndoc
    max_df = float(_pget(params, "maxDF", float(2 ** 63 - 1)))
    min_df = float(_pget(params, "minDF", 1.0))
    max_df = max_df if max_df >= 1.0 else max_df * docs
    min_df = min_df if min_df >= 1.0 else min_df * docs
    if max_df < min_df:
        raise ValueError("MaxDF must be greater than MinDF!")
    # (word count, document frequency) reduced on one owner rank per word, filtered by df there, ordered by
    # count desc / word asc (parallel/sort.merged_vocabulary; DocCountVectorizerTrainBatchOp.java:77 pSort)
    from ...parallel.sort import merged_vocabulary
    merged = merged_vocabulary({k: (wc_c[k], df_c[k]) for k in df_c},
                               keep=lambda w, c: min_df <= c[1] <= max_df)
    keep = [(w, c[0], math.log((1.0 + docs) / (1.0 + c[1]))) for w, c in merged]
    vocab = int(_pget(params, "vocabSize", 2 ** 18))
    keep = keep[:vocab]
    meta = Params().set("minTF", float(_pget(params, "minTF", 1.0))) \
        .set("featureType", _ename(_pget(params, "featureType"), "WORD_COUNT"))
    return SimpleModelDataConverter.rows_from(meta, _tuple3_rows(keep))


def _tuple3_rows(keep) -> List[str]:
    """``gson_dumps(_Tuple3(word, idf, index))`` for every vocabulary entry, with the idf digits from the C++ Java
    double formatter in one call (the generic serializer took ~1 s per 1e5 words)."""
    from ... import _native
    idfs = np.asarray([float(idf) for _, _, idf in keep], dtype=np.float64)
    joined = _native.java_double_join(idfs) if len(keep) else ""
    if joined is None:
        return [gson_dumps(_Tuple3(w, float(idf), i), java_map_order=False) for i, (w, _, idf) in enumerate(keep)]
    ds = joined.split(",") if len(keep) else []
    return ['{"f0":' + _gson_escape(w) + ',"f1":' + d + ',"f2":' + str(i) + '}'
            for i, ((w, _, _), d) in enumerate(zip(keep, ds))]


def _string_block(mt: MTable, col: str, dev):
    """The column as a packed ``StringBlock`` on ``dev`` (a packed column moves as bytes; a list is packed once)."""
    from ...common.strings import StringBlock
    v = mt.col(col).values
    blk = v if isinstance(v, StringBlock) else StringBlock.from_list(mt.column_values(col))
    return blk.to(dev)


def train_doc_hash_count_vectorizer(mt: MTable, params: Params) -> List[tuple]:
    """Hashed word counts over all documents (the reference counts word occurrences, not document
    frequency, in ``HashingTF``), idf ``log((N + 1) / (count + 1))`` for indices with count >= minDF.

    Tensor form (``DocHashCountVectorizerTrainBatchOp.java:40-60`` reduces per-task HashMaps): the documents are
    split on the device (``ops/strings.split_tokens``), every token hashed by the device murmur3
    (``csrc/feature.hip``), counted by ``bincount`` and the ``[numFeatures + 1]`` int64 vector (counts | #docs)
    summed over ranks in ONE all-reduce."""
    from ...ops.strings import murmur3_utf8_index, split_tokens
    from ..feature.encoders import feature_device
    col = params.get("selectedCol")
    nf = int(_pget(params, "numFeatures", 1 << 18))
    dev = feature_device()
    tok, _ = split_tokens(_string_block(mt, col, dev))
    acc = torch.zeros(nf + 1, dtype=torch.int64, device=dev)
    if len(tok):
        acc[:nf] = torch.bincount(murmur3_utf8_index(tok, nf).to(dev), minlength=nf)
    acc[nf] = mt.num_rows                       # COUNT(1): null documents count too
    comm.all_reduce(acc, "sum")
    acc = acc.cpu().numpy()
    cnt, docs = acc[:nf], int(acc[nf])
    min_df = float(_pget(params, "minDF", 1.0))
    min_df = min_df if min_df >= 1.0 else min_df * docs
    keys = np.flatnonzero((cnt > 0) & (cnt >= min_df))
    vals = cnt[keys]
    # Math.log per distinct count (libm, as the per-key form), broadcast to the keys
    uniq, inv = np.unique(vals, return_inverse=True)
    logs = np.asarray([math.log((docs + 1.0) / (float(c) + 1.0)) for c in uniq.tolist()], dtype=np.float64)
    meta = Params().set("numFeatures", nf).set("minTF", float(_pget(params, "minTF", 1.0))) \
        .set("featureType", _ename(_pget(params, "featureType"), "WORD_COUNT"))
    return SimpleModelDataConverter.rows_from(meta, [_int_double_map_json(keys, logs[inv.reshape(-1)])])


def _int_double_map_json(keys: np.ndarray, vals: np.ndarray) -> str:
    """Gson of a ``HashMap<Integer, Double>`` whose keys are below its capacity (the reference's
    ``new HashMap<>(numFeatures)`` over indices < numFeatures): iteration is by bucket = ``k ^ (k >>> 16)``,
    one key per bucket, so the order is ascending in that value whatever the insertion order."""
    from ...common.javafmt import java_double_str
    from ... import _native
    order = np.argsort(keys ^ (keys >> 16), kind="stable")
    k, v = keys[order].tolist(), vals[order]
    body = _native.java_double_join(v) if len(k) else ""
    strs = body.split(",") if body else [java_double_str(float(x)) for x in v.tolist()]
    return "{" + ",".join('"%d":%s' % (a, b) for a, b in zip(k, strs)) + "}"


class _VectorizerMapper(ModelMapper):
    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.col = p.get("selectedCol")
        self.col_idx = find_col_index(dataSchema.names, self.col)
        out = _pget(p, "outputCol") or self.col
        self.helper = OutputColsHelper(dataSchema, [out], [Types.SPARSE_VECTOR], _pget(p, "reservedCols"))

    def _vec(self, content: str):
        raise NotImplementedError

    def _map_row_values(self, row):
        v = row[self.col_idx]
        return [None if v is None else self._vec(str(v))]

    # ---- columnar path: a packed document column, every document's vector from whole-token-array ops
    def _token_features(self, tok):
        """(feature index int64 [T], token counts toward the vector bool [T], idf / value table fp64 [F]) of the
        tokens, or None (the row path)."""
        raise NotImplementedError

    def _map_columns(self, mt):
        from ...common.strings import StringBlock
        col = mt.col(self.col)
        if isinstance(col.values, StringBlock) and col.nulls is None and len(col.values):
            out = self._columnar(col.values)
            if out is not None:
                return [out]
        return super()._map_columns(mt)

    def _columnar(self, blk):
        from ...common.linalg.block import SparseBlock
        from ...ops.strings import split_tokens
        n = len(blk)
        tok, doc = split_tokens(blk)
        dev = doc.device
        ntok = torch.bincount(doc, minlength=n)
        nulls = blk.nulls.to(dev) if blk.nulls is not None else None
        live = ntok if nulls is None else ntok[~nulls]
        if bool((live == 0).any()):
            return None                  # an all-space document: 1 / len(tokens) fails on the row path too
        feats = self._token_features(tok)
        if feats is None:
            return None
        fidx, ok, table = feats
        F = int(self.feature_size)
        key = doc[ok] * F + fidx[ok]
        uk, cnt = torch.unique(key, return_counts=True)          # sorted: by document, then feature index
        d, i = uk // F, uk % F
        nt = ntok.to(torch.float64)[d]
        c = cnt.to(torch.float64)
        min_count = torch.full_like(nt, self.min_tf) if self.min_tf >= 1.0 else self.min_tf * nt
        keep = c >= min_count
        ratio = 1.0 / nt
        idf = table.to(dev)[i]
        ft = self.ftype
        if ft == "IDF":
            val = idf
        elif ft == "WORD_COUNT":
            val = c
        elif ft == "TF_IDF":
            val = idf * c * ratio
        elif ft == "BINARY":
            val = torch.ones_like(c)
        elif ft == "TF":
            val = c * ratio
        else:
            return None
        per = torch.bincount(d[keep], minlength=n)
        crow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(per, 0, out=crow[1:])
        return Column(SparseBlock(crow, i[keep], val[keep], F), nulls)


class DocCountVectorizerModelMapper(_VectorizerMapper):
    def loadModel(self, rows):
        import json
        meta, data = SimpleModelDataConverter.split_rows(rows)
        self.min_tf = float(meta.get("minTF"))
        self.ftype = _ename(meta.get("featureType"), "WORD_COUNT")
        self.vocab = {}
        for s in data:
            d = json.loads(s)
            self.vocab[d["f0"]] = (int(d["f2"]), float(d["f1"]))
        self.n = len(data)
        self.feature_size = self.n

    def _token_features(self, tok):
        """Vocabulary ids through the device dictionary encoding of the tokens: one dict probe per distinct token."""
        from ...ops.strings import unique_ids
        enc = unique_ids(tok)
        if enc is None:
            return None
        ids, rep = enc
        words = tok.take(rep).to_list()
        lut = torch.tensor([self.vocab[w][0] if w in self.vocab else -1 for w in words] or [0], dtype=torch.int64)
        table = torch.zeros(max(self.n, 1), dtype=torch.float64)
        for w, (j, idf) in self.vocab.items():
            table[j] = idf
        fidx = lut.to(ids.device)[ids] if len(words) else ids
        return fidx.clamp(min=0), fidx >= 0, table

    def _vec(self, content):
        toks = java_split(content, WORD_DELIMITER)
        min_count = self.min_tf if self.min_tf >= 1.0 else self.min_tf * len(toks)
        ratio = 1.0 / len(toks)
        cnt = Counter(t for t in toks if t in self.vocab)
        fn = FEATURE_TYPES[self.ftype]
        items = sorted((self.vocab[w][0], fn(self.vocab[w][1], float(c), ratio)) for w, c in cnt.items()
                       if c >= min_count)
        return SparseVector(self.n, [i for i, _ in items], [v for _, v in items])


class DocHashCountVectorizerModelMapper(_VectorizerMapper):
    def loadModel(self, rows):
        import json
        meta, data = SimpleModelDataConverter.split_rows(rows)
        self.nf = int(meta.get("numFeatures"))
        self.min_tf = float(meta.get("minTF"))
        self.ftype = _ename(meta.get("featureType"), "WORD_COUNT")
        self.idf = {int(k): float(v) for k, v in json.loads(data[0]).items()} if data else {}
        self.feature_size = self.nf

    def _token_features(self, tok):
        """Guava murmur3 bucket of every token on the device (empty tokens included, as the row path hashes them);
        the model's idf map as a dense [numFeatures] table and membership mask."""
        from ...ops.strings import murmur3_utf8_index
        idx = murmur3_utf8_index(tok, self.nf)
        table = torch.zeros(max(self.nf, 1), dtype=torch.float64)
        mask = torch.zeros(max(self.nf, 1), dtype=torch.bool)
        if self.idf:
            k = torch.tensor(list(self.idf.keys()), dtype=torch.int64)
            table[k] = torch.tensor(list(self.idf.values()), dtype=torch.float64)
            mask[k] = True
        return idx, mask.to(idx.device)[idx], table

    def _vec(self, content):
        from ..feature.encoders import murmur3_index
        toks = java_split(content, WORD_DELIMITER)
        min_count = self.min_tf if self.min_tf >= 1.0 else self.min_tf * len(toks)
        ratio = 1.0 / len(toks)
        idx = murmur3_index(toks, self.nf).tolist() if toks else []
        cnt = Counter(i for i in idx if i in self.idf)
        fn = FEATURE_TYPES[self.ftype]
        items = sorted((i, fn(self.idf[i], float(c), ratio)) for i, c in cnt.items() if c >= min_count)
        return SparseVector(self.nf, [i for i, _ in items], [v for _, v in items])

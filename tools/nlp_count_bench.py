#!/usr/bin/env python3
"""NLP count training at scale (SURVEY §2.10 DocHashCountVectorizer / DocCountVectorizer): ``--docs`` synthetic
documents of ``--tokens`` words drawn (Zipf-like) from a ``--vocab``-word vocabulary, built directly as a packed
``StringBlock`` on the device, then trained by the public ops.  Prints one JSON line per op with docs/s.

    python tools/nlp_count_bench.py --docs 10000000 --tokens 8 --vocab 100000
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def make_docs(ndoc, ntok, nvocab, dev, seed=0):
    from alink_amd.common.strings import StringBlock
    g = torch.Generator(device="cpu").manual_seed(seed)
    vocab = StringBlock.from_list([f"w{i:x}" + ("é" if i % 7 == 0 else "") for i in range(nvocab)]).to(dev)
    # Zipf-like word ids: floor(nvocab ** u) - 1
    u = torch.rand(ndoc * ntok, generator=g, dtype=torch.float64).to(dev)
    ids = (torch.pow(float(nvocab), u).floor().to(torch.int64) - 1).clamp(0, nvocab - 1)
    toks = vocab.take(ids)                                    # tokens back to back
    tl = toks.lengths().view(ndoc, ntok)
    dl = tl.sum(1) + (ntok - 1)
    doff = torch.zeros(ndoc + 1, dtype=torch.int64, device=dev)
    torch.cumsum(dl, 0, out=doff[1:])
    data = torch.full((int(doff[-1]),), 0x20, dtype=torch.uint8, device=dev)
    # token k of a document starts after the previous tokens and k spaces
    tstart = doff[:-1].view(ndoc, 1) + torch.cumsum(tl, 1) - tl + torch.arange(ntok, device=dev).view(1, ntok)
    lens = tl.reshape(-1)
    seg = torch.repeat_interleave(torch.arange(ndoc * ntok, device=dev), lens)
    j = torch.arange(int(lens.sum()), device=dev) - torch.repeat_interleave(toks.offsets[:-1], lens)
    data[tstart.reshape(-1)[seg] + j] = toks.data
    return StringBlock(data, doff)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--tokens", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ops", default="hash,count")
    a = ap.parse_args()
    from alink_amd import useLocalEnv, DocHashCountVectorizerTrainBatchOp, DocCountVectorizerTrainBatchOp
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = useLocalEnv(1)
    dev = env.device
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    t = time.perf_counter()
    blk = make_docs(a.docs, a.tokens, a.vocab, dev)
    sync()
    t_gen = time.perf_counter() - t
    src = TableSourceBatchOp(MTable(TableSchema(["doc"], [Types.STRING]), [Column(blk)]))
    for name in a.ops.split(","):
        times = []
        for _ in range(a.reps):
            op = (DocHashCountVectorizerTrainBatchOp().setSelectedCol("doc") if name == "hash" else
                  DocCountVectorizerTrainBatchOp().setSelectedCol("doc"))
            sync()
            t = time.perf_counter()
            rows = op.linkFrom(src).collect()
            sync()
            times.append(time.perf_counter() - t)
        tm = sorted(times)[len(times) // 2]
        print(json.dumps({"op": name, "docs": a.docs, "tokens_per_doc": a.tokens, "vocab": a.vocab,
                          "device": str(dev), "s": round(tm, 4), "docs_per_s": a.docs / tm,
                          "tokens_per_s": a.docs * a.tokens / tm, "model_rows": len(rows),
                          "datagen_s": round(t_gen, 2), "all_s": [round(x, 4) for x in times]}), flush=True)


if __name__ == "__main__":
    main()

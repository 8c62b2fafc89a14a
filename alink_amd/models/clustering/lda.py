"""Latent Dirichlet allocation: collapsed-Gibbs "em" and online variational Bayes (reference
``A/operator/batch/clustering/LdaTrainBatchOp.java``, ``A/operator/common/clustering/lda/*``,
``A/operator/common/clustering/{LdaModelData,LdaModelDataConverter,LdaModelMapper}.java``).

Kept from the reference: the vocabulary is a DocCountVectorizer model (``vocabSize`` most frequent words,
stored as ``{"f0":word,"f1":idf,"f2":index}`` rows after the topic matrix); defaults alpha = 50/K + 1,
beta = 1.01 for ``em`` and 1/K for ``online``; ``em`` keeps the ``(V + 1) x K`` word-topic count matrix
``gamma`` (last row = topic totals) and predicts with ``p(w|z) p(z)`` normalised per word; ``online`` keeps
``lambda`` (``K x V``), updated with ``rho = (tau0 + t)^-kappa`` from mini-batches of ``subsamplingRate``
of the corpus, optionally re-estimating alpha by Newton steps (``UpdateLambdaAndAlpha``); the document E-step
iterates ``gamma_d = alpha + e^{E log theta_d} * (sum_w c_w / phinorm_w e^{E log beta_w})`` until the mean
change is below 1e-3 (``LdaUtil.getTopicDistributionMethod``); the model meta records alphaArray,
betaArray, topicNum, vocabularySize, method, logLikelihood and logPerplexity as the reference defines them: for
``em`` the token log-likelihood over -LL / vocabularySize (``EmLogLikelihood``, ``BuildEmLdaModel``), for
``online`` the variational bound (``online_log_likelihood``) over -LL / the last mini-batch's token count
(``OnlineLogLikelihood``, ``BuildOnlineLdaModel``).

Differences: the Gibbs sampler includes the document-topic factor ``(n_dk + alpha)`` of collapsed LDA (the
reference's ``EmCorpusStep`` samples from the word factor only), and sweeps all tokens of a rank in
parallel from the previous sweep's counts (AD-LDA) — a device-wide categorical draw per token followed by
``index_add_`` recounts and one all-reduce of the ``V x K`` counts.  The online E-step runs every document
of the mini-batch at once (token-level gathers + segment sums), with a per-document convergence mask.
"""
from __future__ import annotations

import json
import math
from typing import List, Tuple

import numpy as np
import torch

from ...common.javafmt import gson_dumps
from ...common.linalg import DenseMatrix, DenseVector, VectorUtil
from ...common.mapper import RichModelMapper
from ...common.model.converter import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...ops import lda as lops
from ...parallel import comm
from ..nlp.text import WORD_DELIMITER, java_split, train_doc_count_vectorizer

__all__ = ["train_lda", "LdaModelMapper"]


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


def _dir_exp(x: torch.Tensor) -> torch.Tensor:
    """E[log theta] of Dirichlet rows: digamma(x) - digamma(sum x)."""
    return torch.digamma(x) - torch.digamma(x.sum(-1, keepdim=True))


def _corpus(mt: MTable, col: str, vocab: dict, dev):
    doc_ids, word_ids, counts = [], [], []
    for di, v in enumerate(mt.column_values(col)):
        if v is None:
            continue
        cnt = {}
        for t in java_split(str(v), WORD_DELIMITER):
            if t in vocab:
                cnt[vocab[t]] = cnt.get(vocab[t], 0) + 1
        for w, c in sorted(cnt.items()):
            doc_ids.append(di)
            word_ids.append(w)
            counts.append(float(c))
    n_docs = mt.num_rows
    return (torch.tensor(doc_ids, dtype=torch.long, device=dev), torch.tensor(word_ids, dtype=torch.long, device=dev),
            torch.tensor(counts, dtype=torch.float64, device=dev), n_docs)


def e_step(doc, word, cts, n_docs, expElogbeta_T, alpha, gamma0, max_iter=100, tol=1e-3):
    """Batched document E-step.  expElogbeta_T: [V, K]; gamma0: [D, K].  Returns (gamma, expElogtheta,
    phinorm per token).  On a GPU with K <= 256: the HIP kernel (one wave per document, all iterations in
    registers, ``ops/lda.estep``); elsewhere the vectorised torch loop below."""
    K = expElogbeta_T.shape[1]
    if gamma0.is_cuda and K <= 256 and n_docs > 0 and lops.kernel_supported(gamma0.device):
        return lops.estep(doc, word, cts, n_docs, expElogbeta_T, alpha, gamma0, max_iter, tol)
    gamma = gamma0.clone()
    active = torch.ones(n_docs, dtype=torch.bool, device=gamma.device)
    eb = expElogbeta_T[word]                                  # [T, K]
    for _ in range(max_iter):
        et = torch.exp(_dir_exp(gamma))
        phinorm = (et[doc] * eb).sum(1) + 1e-100
        acc = torch.zeros_like(gamma).index_add_(0, doc, eb * (cts / phinorm)[:, None])
        new = alpha[None, :] + et * acc
        change = (new - gamma).abs().sum(1) / K
        gamma = torch.where(active[:, None], new, gamma)
        active = active & (change > tol)
        if not bool(active.any()):
            break
    et = torch.exp(_dir_exp(gamma))
    phinorm = (et[doc] * eb).sum(1) + 1e-100
    return gamma, et, phinorm


def online_log_likelihood(gamma, doc, word, cts, lam, alpha, beta, task_num: int = 1) -> float:
    """The online-LDA variational bound of ``OnlineLogLikelihood.logLikelihood`` (reference
    A/operator/common/clustering/lda/OnlineLogLikelihood.java:33-70) for documents whose E-step gammas are
    ``gamma`` [D, K] (tokens: ``doc``/``word``/``cts``; ``lam`` [K, V] topic-word Dirichlet, ``alpha`` [K]):
      sum_d [ sum_w c_dw logsumexp_k(E[log theta_dk] + E[log beta_kw]) + sum_k (alpha_k - gamma_dk) E[log theta_dk]
              + sum_k (lgamma(gamma_dk) - lgamma(alpha_k)) + lgamma(sum alpha) - lgamma(sum_k gamma_dk) ]
      + ( sum (beta - lam) E[log beta] + sum (lgamma(lam) - lgamma(beta)) - sum_k (lgamma(sum_v lam_kv)
          - lgamma(beta V)) ) / task_num
    Every rank passes its own documents; the caller sums the returned parts over ranks (each adds 1/task_num of
    the topics part, as the reference's tasks do).  Documents without tokens are skipped (the reference's
    corpus holds none)."""
    K, V = lam.shape
    elog_beta = _dir_exp(lam)                                         # [K, V]
    has = torch.zeros(gamma.shape[0], dtype=torch.bool, device=gamma.device)
    if doc.numel():
        has[doc] = True
    g = gamma[has]
    elog_theta_all = _dir_exp(gamma)
    corpus = 0.0
    if doc.numel():
        tok = torch.logsumexp(elog_theta_all[doc] + elog_beta.T[word], dim=1)
        corpus += float((cts * tok).sum())
    if g.shape[0]:
        et = elog_theta_all[has]
        corpus += float(((alpha[None, :] - g) * et).sum())
        corpus += float((torch.lgamma(g) - torch.lgamma(alpha)[None, :]).sum())
        corpus += float(g.shape[0] * torch.lgamma(alpha.sum()) - torch.lgamma(g.sum(1)).sum())
    topics = float(((beta - lam) * elog_beta).sum() + (torch.lgamma(lam) - math.lgamma(beta)).sum()
                   - (torch.lgamma(lam.sum(1)) - math.lgamma(beta * V)).sum())
    return corpus + topics / task_num


def update_lambda_alpha(lam, alpha, batch, logphat, n_docs_batch: float, t: int, tau0: float, kappa: float,
                        eta: float, rate: float, optimize_alpha: bool):
    """One online step (reference ``UpdateLambdaAndAlpha.calculateLambdaAndAlpha``):
    ``lambda <- (1 - rho) lambda + rho (eta + batch / subSamplingRate)`` with ``rho = (tau0 + t)^-kappa`` and
    ``batch`` = the mini-batch's word-topic statistics times exp(E[log beta]) of the old lambda; then a Newton
    step on alpha from the batch's summed E[log theta] (``logphat``), kept only if every component stays > 0."""
    rho = (tau0 + t) ** (-kappa)
    if n_docs_batch <= 0:
        return lam, alpha
    lam = (1 - rho) * lam + rho * (eta + batch / rate)
    if optimize_alpha:
        B = n_docs_batch
        lp = logphat / B
        gradf = B * (-torch.digamma(alpha) + torch.digamma(alpha.sum()) + lp)
        c = B * torch.polygamma(1, alpha.sum())
        q = -B * torch.polygamma(1, alpha)
        b = (gradf / q).sum() / (1.0 / c + (1.0 / q).sum())
        dalpha = -(gradf - b) / q
        if bool((rho * dalpha + alpha > 0).all()):
            alpha = alpha + rho * dalpha
    return lam, alpha


def _online(doc, word, cts, n_docs, V, K, params, alpha0, eta, seed, dev):
    num_iter = int(_pget(params, "numIter", 10))
    tau0 = float(_pget(params, "onlineLearningOffset", 1024.0))
    kappa = float(_pget(params, "learningDecay", 0.51))
    rate = float(_pget(params, "subsamplingRate", 0.05))
    opt_alpha = bool(_pget(params, "optimizeDocConcentration", True))
    lam = torch.from_numpy(np.random.default_rng(seed).gamma(100.0, 1.0 / 100.0, size=(K, V))).to(dev)
    alpha = torch.full((K,), alpha0, dtype=torch.float64, device=dev)
    rng = np.random.default_rng(seed + 7919 * comm.get_rank())
    last_words = 0.0
    for t in range(1, num_iter + 1):
        pick = rng.random(n_docs) < rate
        if not pick.any() and n_docs:
            pick[rng.integers(0, n_docs)] = True
        sel = torch.as_tensor(pick, device=dev)
        remap = torch.cumsum(sel.long(), 0) - 1
        tok = sel[doc]
        d_b, w_b, c_b = remap[doc[tok]], word[tok], cts[tok]
        nb = int(sel.sum())
        expElogbeta = torch.exp(_dir_exp(lam))                 # [K, V]
        g0 = torch.from_numpy(rng.gamma(100.0, 1.0 / 100.0, size=(nb, K))).to(dev)
        gamma, et, phinorm = e_step(d_b, w_b, c_b, nb, expElogbeta.T, alpha, g0)
        stat = torch.zeros((V, K), dtype=torch.float64, device=dev)
        stat.index_add_(0, w_b, et[d_b] * (c_b / phinorm)[:, None])
        logphat = (_dir_exp(gamma)).sum(0) if nb else torch.zeros(K, dtype=torch.float64, device=dev)
        buf = torch.cat([stat.reshape(-1), logphat,
                         torch.tensor([float(nb), float(c_b.sum()) if nb else 0.0], dtype=torch.float64, device=dev)])
        comm.all_reduce(buf, "sum")
        stat = buf[:V * K].reshape(V, K).T * expElogbeta
        logphat, B, last_words = buf[V * K:V * K + K], float(buf[-2]), float(buf[-1])
        lam, alpha = update_lambda_alpha(lam, alpha, stat, logphat, B, t, tau0, kappa, eta, rate, opt_alpha)
    return lam, alpha, last_words


def _gibbs(doc, word, cts, n_docs, V, K, params, alpha, beta, seed, dev):
    num_iter = int(_pget(params, "numIter", 10))
    reps = cts.long()
    d_tok = torch.repeat_interleave(doc, reps)
    w_tok = torch.repeat_interleave(word, reps)
    g = torch.Generator(device=dev).manual_seed(seed + 7919 * comm.get_rank())
    z = torch.randint(0, K, (d_tok.numel(),), generator=g, device=dev)

    def counts(z):
        # integer histograms (bincount: native int atomics, no fp64 CAS contention on hot words)
        nd = torch.bincount(d_tok * K + z, minlength=max(n_docs, 1) * K).reshape(max(n_docs, 1), K).double()
        nw = torch.bincount(w_tok * K + z, minlength=V * K).reshape(V, K).double()
        comm.all_reduce(nw, "sum")
        return nd, nw

    nd, nw = counts(z)
    use_kernel = lops.kernel_supported(dev)
    for _ in range(num_iter):
        nk = nw.sum(0)
        if use_kernel:
            # K21: per-token topic walk straight from the count tables (same formula, same uniforms)
            u = torch.rand(d_tok.numel(), generator=g, device=dev, dtype=torch.float64)
            z = lops.gibbs_sweep(d_tok, w_tok, z, nd, nw, nk, alpha, beta, V, u)
            nd, nw = counts(z)
            continue
        own = torch.nn.functional.one_hot(z, K).to(torch.float64)
        p = (nd[d_tok] - own + alpha) * (nw[w_tok] - own + beta) / (nk[None, :] - own + V * beta)
        cum = torch.cumsum(p, 1)
        u = torch.rand(d_tok.numel(), generator=g, device=dev, dtype=torch.float64) * cum[:, -1]
        z = torch.searchsorted(cum, u[:, None]).squeeze(1).clamp(max=K - 1)
        nd, nw = counts(z)
    return nd, nw


def train_lda(mt: MTable, params: Params, env) -> List[tuple]:
    dev = env.device
    col = params.get("selectedCol")
    K = int(params.get("topicNum"))
    method = str(getattr(_pget(params, "method", "em"), "name", _pget(params, "method", "em"))).lower()
    seed = int(_pget(params, "randomSeed", 0)) if params.contains("randomSeed") else 0
    dcv = Params().set("selectedCol", col).set("vocabSize", int(_pget(params, "vocabSize", 1 << 18))) \
        .set("featureType", "WORD_COUNT")
    vocab_rows = train_doc_count_vectorizer(mt, dcv)
    vocab_list = [r[1] for r in vocab_rows[1:]]
    vocab = {}
    for s in vocab_list:
        d = json.loads(s)
        vocab[d["f0"]] = int(d["f2"])
    V = len(vocab)
    doc, word, cts, n_docs = _corpus(mt, col, vocab, dev)
    alpha = float(_pget(params, "alpha", -1.0))
    beta = float(_pget(params, "beta", -1.0))
    if method == "online":
        alpha = 1.0 / K if alpha == -1 else alpha
        beta = 1.0 / K if beta == -1 else beta
        lam, alpha_vec, last_words = _online(doc, word, cts, n_docs, V, K, params, alpha, beta, seed, dev)
        topic = lam / lam.sum(1, keepdim=True)
        matrix = DenseMatrix(lam.cpu().numpy())                      # K x V
        alphas = alpha_vec.cpu().numpy().tolist()
        gamma, _, _ = e_step(doc, word, cts, n_docs, torch.exp(_dir_exp(lam)).T, alpha_vec,
                             torch.ones((n_docs, K), dtype=torch.float64, device=dev))
        theta = gamma / gamma.sum(1, keepdim=True)
        m_name = "online"
    else:
        alpha = 50.0 / K + 1 if alpha == -1 else alpha
        beta = 0.01 + 1 if beta == -1 else beta
        nd, nw = _gibbs(doc, word, cts, n_docs, V, K, params, alpha, beta, seed, dev)
        gam = torch.cat([nw, nw.sum(0, keepdim=True)], 0)            # (V + 1) x K
        matrix = DenseMatrix(gam.cpu().numpy())
        alphas = [alpha] * K
        topic = ((nw + beta) / (nw.sum(0) + V * beta)[None, :]).T     # K x V
        theta = (nd + alpha) / (nd + alpha).sum(1, keepdim=True)
        m_name = "em"
    if m_name == "online":
        # the variational bound (OnlineLogLikelihood) over -LL / the last step's sampled token count
        # (BuildOnlineLdaModel.java:66-70)
        part = online_log_likelihood(gamma, doc, word, cts, lam, alpha_vec, beta, comm.get_world_size())
        denom = max(round(last_words), 1)
    else:
        # EmLogLikelihood: sum over tokens of log(theta_d . phi_w), over -LL / vocabularySize
        # (BuildEmLdaModel.java:54-55)
        probs = (theta[doc] * topic.T[word]).sum(1) if doc.numel() else \
            torch.zeros(0, dtype=torch.float64, device=dev)
        part = float((cts * torch.log(probs)).sum()) if doc.numel() else 0.0
        denom = max(V, 1)
    ll = torch.tensor([part], dtype=torch.float64)
    comm.all_reduce(ll, "sum")
    ll = float(ll[0])
    meta = Params().set("logPerplexity", -ll / denom).set("betaArray", [beta] * K) \
        .set("logLikelihood", ll).set("method", m_name).set("alphaArray", alphas).set("topicNum", K) \
        .set("vocabularySize", V)
    data = [gson_dumps(matrix, java_map_order=False)] + vocab_list
    return SimpleModelDataConverter.rows_from(meta, data)


class LdaModelMapper(RichModelMapper):
    def predResultType(self):
        return Types.LONG

    def loadModel(self, rows):
        meta, data = SimpleModelDataConverter.split_rows(rows)
        self.K = int(meta.get("topicNum"))
        self.V = int(meta.get("vocabularySize"))
        method = str(getattr(meta.get("method"), "name", meta.get("method"))).lower()
        m = json.loads(data[0])
        mat = np.asarray(m["data"], dtype=np.float64).reshape(int(m["n"]), int(m["m"])).T
        self.alpha = np.asarray(meta.get("alphaArray"), dtype=np.float64)
        beta = np.asarray(meta.get("betaArray"), dtype=np.float64)
        if method == "em":                                    # LdaModelMapper.getWordTopicMatrixGibbs
            V, K = self.V, self.K
            tot = mat[V]
            pz = tot / tot.sum()
            pwz = (mat[:V] + beta[None, :]) / (tot[None, :] + K * beta[None, :]) * pz[None, :]
            s = pwz.sum(1, keepdims=True)
            pwz = np.where(s != 0, pwz / np.where(s == 0, 1, s), pwz)
            wt = np.minimum(pwz, 1.0).T                        # K x V
        else:
            wt = mat
        wt_t = torch.as_tensor(wt)
        self.expElogbeta_T = torch.exp(_dir_exp(wt_t)).T       # V x K
        self.vocab = {}
        for s in data[1:]:
            d = json.loads(s)
            self.vocab[d["f0"]] = int(d["f2"])

    def _map_row_values(self, row):
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        return [c.to_list()[0] for c in self._map_columns(mt)]

    def _map_columns(self, mt):
        col = self.params.get("selectedCol")
        doc, word, cts, n = _corpus(mt, col, self.vocab, torch.device("cpu"))
        g0 = torch.from_numpy(np.random.default_rng(0).gamma(100.0, 100.0, size=(n, self.K)))
        gamma, _, _ = e_step(doc, word, cts, n, self.expElogbeta_T, torch.as_tensor(self.alpha), g0)
        has = torch.zeros(n, dtype=torch.bool).index_fill_(0, doc, True) if doc.numel() else torch.zeros(n, dtype=torch.bool)
        vals = torch.where(has[:, None], gamma, torch.zeros_like(gamma)).numpy()
        preds, details = [], []
        for v in vals:
            s = np.abs(v).sum()
            dv = v / s if s > 0 else v
            preds.append(int(np.argmax(v)) if s > 0 else 0)
            details.append(VectorUtil.toString(DenseVector(dv)))
        cols = [Column.from_values(preds, Types.LONG)]
        if self.detail_col:
            cols.append(Column.from_values(details, Types.STRING))
        return cols

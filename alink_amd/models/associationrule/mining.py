"""Frequent-pattern mining: FP-Growth (itemsets + association rules) and PrefixSpan (sequential patterns +
sequence rules).

Reference: ``A/operator/batch/associationrule/FpGrowthBatchOp.java`` (item order = support desc, name asc
:153-178; min support count = ``floor(N * percent)`` unless given :268-281; pattern strings in item-index
order :283-320), ``A/operator/common/associationrule/{ParallelFpGrowth,FpTree,AssociationRule}.java``
(rules: ``lift = supXY*N/(supX*supY)``, ``lift >= minLift && confidence >= minConfidence``),
``PrefixSpanBatchOp.java`` (item support counted per occurrence :104-139, sequences encoded with 0 between
elements :166-203, ``encodeSequence`` :273-293), ``ParallelPrefixSpan.java``, ``SequenceRule.java``
(antecedent = all but the last element, consequent = last element).

Parallel scheme (PFP): transactions/sequences are encoded once, identical ones are de-duplicated with
counts, and the distinct encoded database is shared; rank r mines the patterns whose *last* item (FP-Growth:
the least frequent item of the pattern; PrefixSpan: the first item) belongs to its item group, and the
pattern lists are all-gathered — the same partition-by-item decomposition as the reference's parallel
FP-growth, with no pattern mined twice.
"""
from __future__ import annotations

import math
from collections import Counter, defaultdict
from typing import Dict, List, Sequence, Tuple

from ...parallel import comm

__all__ = ["fp_growth", "association_rules", "prefix_span", "sequence_rules"]


def _min_support(n: int, count: int, percent: float) -> int:
    return int(count) if count is not None and count >= 0 else int(math.floor(n * percent))


# ---------------------------------------------------------------------------------------------------
# FP-Growth
# ---------------------------------------------------------------------------------------------------
def _mine(db: List[Tuple[Tuple[int, ...], int]], suffix: Tuple[int, ...], min_sup: int, max_len: int,
          out: Dict[Tuple[int, ...], int], allowed_last=None):
    """Conditional-pattern-base recursion.  ``db`` holds (sorted item tuple, count); patterns grow by
    prepending items that precede the current suffix in the global order."""
    counts = Counter()
    for items, c in db:
        for it in items:
            counts[it] += c
    for it, c in counts.items():
        if c < min_sup:
            continue
        if allowed_last is not None and it not in allowed_last:
            continue
        pat = (it,) + suffix
        out[pat] = c
        if len(pat) >= max_len:
            continue
        cond = []
        for items, cc in db:
            if it in items:
                pre = items[:items.index(it)]
                if pre:
                    cond.append((pre, cc))
        if cond:
            _mine(cond, pat, min_sup, max_len, out)


def fp_growth(transactions: Sequence[Sequence[str]], min_support_count: int, min_support_percent: float,
              max_pattern_length: int):
    """Returns (item names by index, patterns {sorted index tuple: support}, N, item supports)."""
    local_counts = Counter()
    local_tx = Counter()
    for t in transactions:
        s = frozenset(t)
        local_tx[s] += 1
        for it in s:
            local_counts[it] += 1
    counts = Counter()
    for c in comm.all_gather_object(dict(local_counts)):
        counts.update(c)
    n = sum(comm.all_gather_object(len(transactions)))
    min_sup = _min_support(n, min_support_count, min_support_percent)
    qualified = [(it, c) for it, c in counts.items() if c >= min_sup]
    qualified.sort(key=lambda t: (-t[1], t[0]))
    names = [it for it, _ in qualified]
    index = {it: i for i, it in enumerate(names)}
    db_counter = Counter()
    for part in comm.all_gather_object([(sorted(index[i] for i in s if i in index), c) for s, c in local_tx.items()]):
        for items, c in part:
            if items:
                db_counter[tuple(items)] += c
    db = list(db_counter.items())
    ws, r = comm.get_world_size(), comm.get_rank()
    mine = {i for i in range(len(names)) if i % ws == r}
    out: Dict[Tuple[int, ...], int] = {}
    _mine(db, (), min_sup, max_pattern_length, out, allowed_last=mine)
    patterns: Dict[Tuple[int, ...], int] = {}
    for part in comm.all_gather_object(out):
        patterns.update(part)
    return names, patterns, n, {index[it]: c for it, c in qualified}


def association_rules(patterns: Dict[Tuple[int, ...], int], n: int, min_confidence: float, min_lift: float,
                      max_consequent_length: int):
    """(antecedent, consequent, support count, lift, support, confidence) for every rule passing the filters."""
    rules = []
    if max_consequent_length <= 0:
        return rules
    for pat, sup_xy in patterns.items():
        if len(pat) < 2:
            continue
        k = len(pat)
        for size in range(1, min(max_consequent_length, k - 1) + 1):
            from itertools import combinations
            for cons in combinations(pat, size):
                ante = tuple(i for i in pat if i not in cons)
                sup_x = patterns.get(ante)
                sup_y = patterns.get(tuple(cons))
                if not sup_x or not sup_y:
                    continue
                conf = sup_xy / sup_x
                lift = sup_xy * n / (sup_x * sup_y)
                if lift >= min_lift and conf >= min_confidence:
                    rules.append((ante, tuple(cons), sup_xy, lift, sup_xy / n, conf))
    return rules


# ---------------------------------------------------------------------------------------------------
# PrefixSpan (itemset elements; sequence / itemset extensions)
# ---------------------------------------------------------------------------------------------------
def _project(db, item, extend_element: bool):
    """Project each (sequence, count, position) on ``item``.

    A position is (element index, item offset) of the last matched item.  Itemset extension (``_item``)
    looks for ``item`` later in the same element; sequence extension looks in later elements."""
    out = []
    for seq, c, pos in db:
        found = None
        if extend_element:
            # the element that holds the last matched item, or a later element containing the whole last
            # pattern element plus the item
            e, off = pos
            el = seq[e]
            for k in range(off + 1, len(el)):
                if el[k] == item:
                    found = (e, k)
                    break
        else:
            e = pos[0] + 1 if pos is not None else 0
            for ee in range(e, len(seq)):
                el = seq[ee]
                if item in el:
                    found = (ee, el.index(item))
                    break
        if found is not None:
            out.append((seq, c, found))
    return out


def _support(db) -> int:
    return sum(c for _, c, _ in db)


def _span(db, pattern, last_element, min_sup, max_len, out):
    """``pattern`` is a tuple of elements (sorted tuples); ``db`` the sequences projected on it."""
    n_items = sum(len(e) for e in pattern)
    if n_items >= max_len:
        return
    seq_ext = Counter()
    item_ext = Counter()
    for seq, c, pos in db:
        e, off = pos
        seen_s, seen_i = set(), set()
        for ee in range(e + 1, len(seq)):
            for it in seq[ee]:
                seen_s.add(it)
        for k in range(off + 1, len(seq[e])):
            seen_i.add(seq[e][k])
        # itemset extension also when a later element contains the whole last element plus the item
        last = set(last_element)
        for ee in range(e + 1, len(seq)):
            el = seq[ee]
            if last.issubset(el):
                mx = max(last)
                for it in el:
                    if it > mx:
                        seen_i.add(it)
        for it in seen_s:
            seq_ext[it] += c
        for it in seen_i:
            item_ext[it] += c
    for it, c in sorted(item_ext.items()):
        if c < min_sup:
            continue
        new_last = tuple(last_element) + (it,)
        pat = pattern[:-1] + (new_last,)
        proj = []
        for seq, cc, pos in db:
            e, off = pos
            found = None
            for k in range(off + 1, len(seq[e])):
                if seq[e][k] == it:
                    found = (e, k)
                    break
            if found is None:
                for ee in range(e + 1, len(seq)):
                    if set(new_last).issubset(seq[ee]):
                        found = (ee, seq[ee].index(it))
                        break
            if found is not None:
                proj.append((seq, cc, found))
        out[pat] = _support(proj)
        _span(proj, pat, new_last, min_sup, max_len, out)
    for it, c in sorted(seq_ext.items()):
        if c < min_sup:
            continue
        pat = pattern + ((it,),)
        proj = _project(db, it, False)
        out[pat] = _support(proj)
        _span(proj, pat, (it,), min_sup, max_len, out)


def prefix_span(sequences: Sequence[Sequence[Sequence[str]]], min_support_count: int, min_support_percent: float,
                max_pattern_length: int):
    """Returns (item names, index 1.., patterns {tuple of element tuples: support}, N)."""
    occ = Counter()
    local = Counter()
    for s in sequences:
        for el in s:
            for it in el:
                occ[it] += 1
        local[tuple(tuple(el) for el in s)] += 1
    counts = Counter()
    for c in comm.all_gather_object(dict(occ)):
        counts.update(c)
    n = sum(comm.all_gather_object(len(sequences)))
    min_sup = _min_support(n, min_support_count, min_support_percent)
    qualified = [(it, c) for it, c in counts.items() if c >= min_sup]
    qualified.sort(key=lambda t: (-t[1], t[0]))
    names = [None] + [it for it, _ in qualified]
    index = {it: i + 1 for i, (it, _) in enumerate(qualified)}
    db_counter = Counter()
    for part in comm.all_gather_object(list(local.items())):
        for s, c in part:
            enc = []
            for el in s:
                ids = sorted({index[i] for i in el if i in index})
                if ids:
                    enc.append(tuple(ids))
            if enc:
                db_counter[tuple(enc)] += c
    db0 = list(db_counter.items())
    ws, r = comm.get_world_size(), comm.get_rank()
    out = {}
    for it in range(1, len(names)):
        if (it - 1) % ws != r:
            continue
        proj = _project([(s, c, None) for s, c in db0], it, False)
        sup = _support(proj)
        if sup < min_sup:
            continue
        pat = ((it,),)
        out[pat] = sup
        _span(proj, pat, (it,), min_sup, max_pattern_length, out)
    patterns = {}
    for part in comm.all_gather_object(out):
        patterns.update(part)
    return names, patterns, n


def sequence_rules(patterns, n: int, min_confidence: float):
    """(antecedent elements, consequent element, support count, support, confidence)."""
    out = []
    for pat, sup_xy in patterns.items():
        if len(pat) <= 1:
            continue
        ante, cons = pat[:-1], pat[-1]
        sup_x = patterns.get(ante)
        if not sup_x:
            continue
        conf = sup_xy / sup_x
        if conf >= min_confidence:
            out.append((ante, (cons,), sup_xy, sup_xy / n, conf))
    return out

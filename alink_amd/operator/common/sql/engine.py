"""Relational operations on (full) ``MTable``s used by the SQL-sugar operators.

Reference: ``A/operator/common/sql/BatchSqlOperators.java:51-388`` (select, as, where/filter, distinct,
orderBy with limit/offset/fetch, groupBy, inner/left/right/full joins over aliases ``a``/``b``, union(All),
intersect(All), minus(All)).
"""
from __future__ import annotations

from collections import Counter, OrderedDict
from typing import Any, List, Optional, Sequence, Tuple

from ....common.table import MTable, Row, infer_type
from ....common.types import AlinkType, TableSchema, Types
from .expr import Expr, compile_expr, parse_expr, parse_select_list, split_top_level

__all__ = ["sql_select", "sql_where", "sql_as", "sql_distinct", "sql_order_by", "sql_group_by", "sql_join",
           "sql_union", "sql_intersect", "sql_minus"]


def _resolver(names: Sequence[str], qualifiers: Optional[dict] = None):
    names = list(names)
    lower = [n.lower() for n in names]

    def resolve(n: str) -> int:
        if qualifiers and "." in n:
            q, c = n.split(".", 1)
            if q in qualifiers:
                off, sub = qualifiers[q]
                if c in sub:
                    return off + sub.index(c)
                sl = [x.lower() for x in sub]
                if c.lower() in sl:
                    return off + sl.index(c.lower())
                raise ValueError(f"Column {n} not found")
        if n in names:
            return names.index(n)
        if n.lower() in lower:
            return lower.index(n.lower())
        if "." in n:
            return resolve(n.split(".", 1)[1])
        raise ValueError(f"Column '{n}' not found in table, all columns: {names}")
    return resolve


def _out_type(e: Expr, schema: TableSchema, vals: List[Any], resolve) -> AlinkType:
    if e.kind == "col":
        return schema.types[resolve(e.args[0])]
    if e.kind == "agg" and e.args[0] == "COUNT":
        return Types.LONG
    if e.kind == "agg" and e.args[0] in ("MIN", "MAX", "SUM") and e.args[1] and e.args[1][0].kind == "col":
        return schema.types[resolve(e.args[1][0].args[0])]
    if e.kind == "cast":
        from ....common.types import type_from_str
        try:
            return type_from_str(e.args[1])
        except ValueError:
            pass
    if e.kind in ("cmp", "and", "or", "not", "isnull", "like", "in", "between"):
        return Types.BOOLEAN
    for v in vals:
        if v is not None:
            return infer_type(v)
    return Types.STRING


def _expand_star(items, schema):
    out = []
    for it in items:
        if it.expr.kind == "star":
            for n in schema.names:
                from .expr import SelectItem
                out.append(SelectItem(Expr("col", n), None, n))
        else:
            out.append(it)
    return out


def _names_for(items):
    names = []
    for i, it in enumerate(items):
        if it.alias:
            names.append(it.alias)
        elif it.expr.kind == "col":
            names.append(it.expr.args[0].split(".")[-1])
        else:
            names.append(f"EXPR${i}")
    return names


def _select_rows(rows: List[Row], schema: TableSchema, clause: str, qualifiers=None) -> Tuple[List[Row], TableSchema]:
    items = _expand_star(parse_select_list(clause), schema)
    resolve = _resolver(schema.names, qualifiers)
    fns = [compile_expr(it.expr, resolve) for it in items]
    out = [Row(tuple(f(r) for f in fns)) for r in rows]
    names = _names_for(items)
    types = [_out_type(it.expr, schema, [o[j] for o in out[:100]], resolve) for j, it in enumerate(items)]
    return out, TableSchema(names, types)


def sql_select(mt: MTable, clause: str, qualifiers: Optional[dict] = None) -> MTable:
    items = _expand_star(parse_select_list(clause), mt.schema)
    resolve = _resolver(mt.schema.names, qualifiers)
    # pure column projection: keep native column storage (tensors stay on device)
    if all(it.expr.kind == "col" for it in items):
        idx = [resolve(it.expr.args[0]) for it in items]
        names = _names_for(items)
        return MTable(TableSchema(names, [mt.schema.types[i] for i in idx]), [mt.cols[i] for i in idx],
                      mt.replicated)
    cols = _select_columnar(mt, items, resolve)
    if cols is not None:
        return cols
    rows, schema = _select_rows(mt.rows(), mt.schema, clause, qualifiers)
    return MTable.from_rows(rows, schema, mt.replicated)


def _select_columnar(mt: MTable, items, resolve=None) -> Optional[MTable]:
    """Whole-column evaluation of a projection (``vexpr``) when every item is a column or a columnar
    expression; None -> the row path."""
    from ....common.table import Column
    from .vexpr import try_evaluate
    if mt.num_rows == 0 or any(it.expr.has_agg() for it in items):
        return None
    resolve = resolve or _resolver(mt.schema.names)
    cols, types = [], []
    for it in items:
        if it.expr.kind == "col":
            i = resolve(it.expr.args[0])
            cols.append(mt.cols[i])
            types.append(mt.schema.types[i])
            continue
        if it.expr.kind == "fn" and it.expr.args[0] in _STRING_FNS:
            sb = _string_columnar(it.expr, mt, resolve)
            if sb is not None:
                cols.append(Column(sb))
                types.append(Types.STRING)
                continue
        r = try_evaluate(it.expr, mt, resolve)
        if r is None:
            return None
        vals, nulls = r
        sample = Column(vals[:100].cpu(), None if nulls is None else nulls[:100].cpu()).to_list()
        t = _out_type(it.expr, mt.schema, sample, resolve)
        if t.torch_dtype is not None and vals.dtype != t.torch_dtype:
            vals = vals.to(t.torch_dtype)
        cols.append(Column(vals, nulls if nulls is not None and bool(nulls.any()) else None))
        types.append(t)
    return MTable(TableSchema(_names_for(items), types), cols, mt.replicated)


_STRING_FNS = ("UPPER", "LOWER", "CONCAT")


def _string_columnar(e, mt: MTable, resolve):
    """UPPER / LOWER / CONCAT over packed string columns and string literals as byte operations on the device
    (``StringBlock`` in, ``StringBlock`` out, NULL in -> NULL out as the row functions); None -> the row path
    (other argument kinds, or non-ASCII text under UPPER / LOWER, whose Unicode case rules the bytes lack)."""
    import torch
    from ....common.strings import StringBlock
    n = mt.num_rows
    if e.kind == "lit":
        return e.args[0].encode("utf-8") if isinstance(e.args[0], str) else None
    if e.kind == "col":
        i = resolve(e.args[0])
        v = mt.cols[i].values
        if not isinstance(v, StringBlock) or mt.schema.types[i] != Types.STRING:
            return None
        return v
    if e.kind != "fn" or e.args[0] not in _STRING_FNS:
        return None
    name, args = e.args[0], [_string_columnar(a, mt, resolve) for a in e.args[1]]
    if any(a is None for a in args):
        return None
    if name in ("UPPER", "LOWER"):
        if len(args) != 1 or not isinstance(args[0], StringBlock):
            return None
        b = args[0]
        if b.data.numel() and bool((b.data >= 0x80).any()):
            return None
        lo, hi = (0x61, 0x7A) if name == "UPPER" else (0x41, 0x5A)
        hit = (b.data >= lo) & (b.data <= hi)
        return StringBlock(torch.where(hit, b.data - 32 if name == "UPPER" else b.data + 32, b.data), b.offsets,
                           b.nulls)
    blocks = [a for a in args if isinstance(a, StringBlock)]
    if not blocks:
        return None
    dev = blocks[0].device
    nulls = None
    lens = []
    for a in args:
        if isinstance(a, StringBlock):
            if a.nulls is not None:
                nm = a.nulls.to(dev)
                nulls = nm if nulls is None else (nulls | nm)
            o = a.offsets.to(dev, torch.int64)
            lens.append(o[1:] - o[:-1])
        else:
            lens.append(torch.full((n,), len(a), dtype=torch.int64, device=dev))
    if nulls is not None:
        lens = [torch.where(nulls, torch.zeros_like(L), L) for L in lens]
    tot = torch.stack(lens).sum(0)
    out_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(tot, 0, out=out_off[1:])
    out = torch.empty(int(out_off[-1]), dtype=torch.uint8, device=dev)
    start = out_off[:-1].clone()
    rows = torch.arange(n, device=dev)
    for a, L in zip(args, lens):
        m = int(L.sum())
        if m:
            row = torch.repeat_interleave(rows, L)
            first = torch.cumsum(L, 0) - L
            k = torch.arange(m, device=dev) - first[row]
            if isinstance(a, StringBlock):
                src = a.data.to(dev)[a.offsets.to(dev, torch.int64)[:-1][row] + k]
            else:
                src = torch.tensor(list(a), dtype=torch.uint8, device=dev)[k]
            out[start[row] + k] = src
        start += L
    return StringBlock(out, out_off, nulls if nulls is not None and bool(nulls.any()) else None)


def sql_as(mt: MTable, clause: str) -> MTable:
    names = [x.strip() for x in split_top_level(clause)]
    if len(names) != len(mt.schema.names):
        raise ValueError("The number of alias names must equal the number of columns")
    return mt.rename(names)


def sql_where(mt: MTable, clause: str) -> MTable:
    e = parse_expr(clause)
    if mt.num_rows and not e.has_agg():
        from .vexpr import try_evaluate
        r = try_evaluate(e, mt, _resolver(mt.schema.names))
        if r is not None and r[0].dtype == __import__("torch").bool:
            keep = r[0] if r[1] is None else (r[0] & ~r[1])      # only TRUE rows survive (NULL drops)
            return mt.take(keep)
    f = compile_expr(e, _resolver(mt.schema.names))
    keep = [i for i, r in enumerate(mt.rows()) if f(r) is True]
    return mt.take(keep)


def _key(v):
    from ....common.linalg import Vector, VectorUtil
    return VectorUtil.toString(v) if isinstance(v, Vector) else v


def sql_distinct(mt: MTable) -> MTable:
    import torch
    if mt.num_rows:
        dev = next((c.values.device for c in mt.cols if isinstance(c.values, torch.Tensor)), torch.device("cpu"))
        code = _row_codes(mt, range(len(mt.cols)), dev)
        if code is not None:
            # first occurrence of every distinct row, in row order (columnar: no per-row tuples)
            first = _first_index(code, int(code.max()) + 1)
            return mt.take(torch.sort(first)[0])
    seen = set()
    keep = []
    for i, r in enumerate(mt.rows()):
        k = tuple(_key(v) for v in r)
        if k not in seen:
            seen.add(k)
            keep.append(i)
    return mt.take(keep)


def sql_order_by(mt: MTable, clause: str, order: str = "asc", limit=None, offset=None, fetch=None) -> MTable:
    keys = []
    for part in split_top_level(clause):
        toks = part.split()
        asc = order.lower() != "desc"
        if len(toks) > 1 and toks[-1].lower() in ("asc", "desc"):
            asc = toks[-1].lower() == "asc"
            part = " ".join(toks[:-1])
        keys.append((parse_expr(part), asc))
    idx = _order_columnar(mt, keys)
    if idx is not None:
        lo = offset if offset is not None and offset > 0 else 0
        idx = idx[lo:]
        if fetch is not None and fetch >= 0:
            idx = idx[:fetch]
        if limit is not None and limit >= 0:
            idx = idx[:limit]
        return mt.take(idx)
    keys = [(compile_expr(e, _resolver(mt.schema.names)), asc) for e, asc in keys]
    rows = mt.rows()
    idx = list(range(len(rows)))
    for f, asc in reversed(keys):
        vals = [f(rows[i]) for i in range(len(rows))]
        # NULLs first in ascending order (Flink default), last in descending
        idx.sort(key=lambda i: (vals[i] is not None, vals[i] if vals[i] is not None else 0), reverse=not asc)
    if offset is not None and offset > 0:
        idx = idx[offset:]
    if fetch is not None and fetch >= 0:
        idx = idx[:fetch]
    if limit is not None and limit >= 0:
        idx = idx[:limit]
    return mt.take(idx)


def _order_columnar(mt: MTable, keys):
    """Row order of ``ORDER BY`` over numeric key expressions evaluated on tensors: stable sorts from the last
    key to the first, NULLs first ascending / last descending (the row path's key), equal keys in input order.
    None (the row path) for a non-columnar key or a NaN key."""
    import torch
    from .vexpr import try_evaluate
    n = mt.num_rows
    if n == 0:
        return None
    res = _resolver(mt.schema.names)
    ev = []
    for e, asc in keys:
        r = try_evaluate(e, mt, res)
        if r is None:
            return None
        v, nm = r
        if not isinstance(v, torch.Tensor) or v.dim() != 1 or v.numel() != n or v.is_complex():
            return None
        if v.dtype == torch.bool:
            v = v.to(torch.int8)
        elif v.is_floating_point():
            if bool(torch.isnan(v if nm is None else v[~nm.to(v.device)]).any()):
                return None
            v = v + 0.0                               # -0.0 == 0.0 for the sort, as for python's compare
        ev.append((v, None if nm is None else nm.to(v.device), asc))
    idx = torch.arange(n, device=ev[0][0].device)
    for v, nm, asc in reversed(ev):
        idx = idx.to(v.device)
        if nm is None:
            idx = idx[torch.sort(v[idx], stable=True, descending=not asc).indices]
            continue
        knm = nm[idx]
        nl, nn = idx[knm], idx[~knm]
        nn = nn[torch.sort(v[nn], stable=True, descending=not asc).indices]
        idx = torch.cat([nl, nn]) if asc else torch.cat([nn, nl])
    return idx.cpu()


def _factorize(c) -> Tuple[Any, int]:
    """(int64 codes [n] on the column's device, number of codes) of one key column; NULL -> its own code."""
    import torch
    v = c.values
    if isinstance(v, torch.Tensor) and v.dim() == 1:
        uniq, inv = torch.unique(v, return_inverse=True)
        k = int(uniq.numel())
        if c.nulls is not None:
            inv = torch.where(c.nulls.to(inv.device), torch.full_like(inv, k), inv)
            k += 1
        return inv.to(torch.int64), k
    from ....common.strings import StringBlock
    if isinstance(v, StringBlock) and len(v):
        # packed strings: the device dictionary encoding (exact, or None on a hash collision -> the list path)
        from ....ops.strings import unique_ids
        enc = unique_ids(v)
        if enc is not None:
            ids, rep = enc
            k = int(rep.numel())
            nm = v.nulls
            if c.nulls is not None:
                cn = c.nulls.to(ids.device)
                nm = cn if nm is None else (nm.to(ids.device) | cn)
            if nm is not None:
                ids = torch.where(nm.to(ids.device), torch.full_like(ids, k), ids)
                k += 1
            return ids, k
    vals = c.to_list()
    if not all(x is None or isinstance(x, (str, int, float, bool)) for x in vals):
        return None, 0
    codes, table = [], {}
    for x in vals:
        codes.append(table.setdefault(_key(x), len(table)))
    return torch.tensor(codes, dtype=torch.int64), len(table)


def _row_codes(mt: MTable, idx, dev):
    """Dense int64 code per row of the column tuple ``idx`` (equal tuples <-> equal codes), or None."""
    import torch
    code = torch.zeros(mt.num_rows, dtype=torch.int64, device=dev)
    for i in idx:
        ci, k = _factorize(mt.cols[i])
        if ci is None:
            return None
        code = torch.unique(code * k + ci.to(dev), return_inverse=True)[1]     # stays < n: no overflow
    return code


def _first_index(code, G: int):
    """[G] first row index of every code value (codes dense in [0, G)), from one stable sort (no atomics)."""
    import torch
    o = torch.argsort(code, stable=True)
    cnt = torch.bincount(code, minlength=G)
    starts = torch.cumsum(cnt, 0) - cnt
    return o[starts]


def _group_by_columnar(mt: MTable, by: str, select: str) -> Optional[MTable]:
    """GROUP BY plain key columns with COUNT / SUM / AVG / MIN / MAX over numeric tensor columns, evaluated per
    column: key codes -> group ids in first-appearance order (the row path's OrderedDict order), then
    bincount / index_add / scatter_reduce over the rows.  None -> the row path."""
    import torch
    from ....common.table import Column
    if mt.num_rows == 0:
        return None
    resolve = _resolver(mt.schema.names)
    keys = [parse_expr(p) for p in split_top_level(by)]
    if any(k.kind != "col" for k in keys):
        return None
    kidx = [resolve(k.args[0]) for k in keys]
    items = _expand_star(parse_select_list(select), mt.schema)
    for it in items:
        e = it.expr
        if e.kind == "col":
            if resolve(e.args[0]) not in kidx:
                return None
        elif e.kind == "agg":
            name, args, distinct = e.args
            if distinct or name not in ("COUNT", "SUM", "AVG", "MIN", "MAX") or len(args) != 1:
                return None
            if args[0].kind == "star":
                if name != "COUNT":
                    return None
            elif args[0].kind != "col":
                return None
            else:
                c = mt.cols[resolve(args[0].args[0])]
                if not (isinstance(c.values, torch.Tensor) and c.values.dim() == 1 and c.values.dtype != torch.bool):
                    return None
        else:
            return None
    n = mt.num_rows
    dev = next((c.values.device for c in mt.cols if isinstance(c.values, torch.Tensor)), torch.device("cpu"))
    gid = _row_codes(mt, kidx, dev)
    if gid is None:
        return None
    G = int(gid.max()) + 1
    first = _first_index(gid, G)
    order = torch.argsort(first)                      # groups in first-appearance order
    rank = torch.empty_like(order)
    rank[order] = torch.arange(G, device=dev)
    g = rank[gid]                                     # group index per row, first-appearance numbering
    firsts = first[order]
    cols, types = [], []
    for it in items:
        e = it.expr
        if e.kind == "col":
            i = resolve(e.args[0])
            cols.append(mt.cols[i].take(firsts.cpu() if not isinstance(mt.cols[i].values, torch.Tensor) else firsts))
            types.append(mt.schema.types[i])
            continue
        name, args, _ = e.args
        if args[0].kind == "star":
            cnt = torch.bincount(g, minlength=G)
            cols.append(Column(cnt))
            types.append(Types.LONG)
            continue
        c = mt.cols[resolve(args[0].args[0])]
        v = c.values.to(dev)
        ok = ~c.nulls.to(dev) if c.nulls is not None else torch.ones(n, dtype=torch.bool, device=dev)
        cnt = torch.bincount(g[ok], minlength=G)
        empty = cnt == 0
        if name == "COUNT":
            cols.append(Column(cnt))
            types.append(Types.LONG)
            continue
        isint = not v.dtype.is_floating_point
        # segmented reductions over the rows sorted (stably) by group: no atomics on a handful of hot group
        # addresses, and the summation order is the row order within each group (the row path's)
        gg = g[ok]
        o = torch.argsort(gg, stable=True)
        vv = v.to(torch.int64 if isint else torch.float64)[ok][o]
        if name in ("SUM", "AVG"):
            if isint:
                cs = torch.zeros(vv.numel() + 1, dtype=torch.int64, device=dev)
                torch.cumsum(vv, 0, out=cs[1:])
                ends = torch.cumsum(cnt, 0)
                acc = cs[ends] - cs[ends - cnt]
            else:
                acc = torch.segment_reduce(vv, "sum", lengths=cnt)
            res = acc if name == "SUM" else acc.to(torch.float64) / cnt.clamp(min=1)
        else:
            res = torch.segment_reduce(vv.to(torch.float64), "min" if name == "MIN" else "max", lengths=cnt)
            res = torch.where(empty, torch.zeros_like(res), res)
            if isint:
                res = res.to(torch.int64)
        nulls = empty if bool(empty.any()) else None
        col = Column(res, nulls)
        t = _out_type(e, mt.schema, col.take(slice(0, 100)).to_list(), resolve)
        if t.torch_dtype is not None and res.dtype != t.torch_dtype:
            col = Column(res.to(t.torch_dtype), nulls)
        cols.append(col)
        types.append(t)
    return MTable(TableSchema(_names_for(items), types), cols)


def sql_group_by(mt: MTable, by: str, select: str) -> MTable:
    out = _group_by_columnar(mt, by, select)
    if out is not None:
        return out
    resolve = _resolver(mt.schema.names)
    kfs = [compile_expr(parse_expr(p), resolve) for p in split_top_level(by)]
    groups: "OrderedDict[tuple, List[Row]]" = OrderedDict()
    for r in mt.rows():
        k = tuple(_key(f(r)) for f in kfs)
        groups.setdefault(k, []).append(r)
    items = _expand_star(parse_select_list(select), mt.schema)
    fns = [compile_expr(it.expr, resolve) for it in items]
    out = [Row(tuple(f(g[0], g) for f in fns)) for g in groups.values()]
    names = _names_for(items)
    types = [_out_type(it.expr, mt.schema, [o[j] for o in out[:100]], resolve) for j, it in enumerate(items)]
    return MTable.from_rows(out, TableSchema(names, types))


def _split_and(e: Expr) -> List[Expr]:
    if e.kind == "and":
        return _split_and(e.args[0]) + _split_and(e.args[1])
    return [e]


_BLOCKED_JOIN_MAX_PAIRS = 1 << 34      # columnar nested-loop joins up to this many pairs (then the hash / row path)


def sql_join(left: MTable, right: MTable, predicate: str, select: str = "*", how: str = "inner") -> MTable:
    ln, rn = left.schema.names, right.schema.names
    qual = {"a": (0, ln), "b": (len(ln), rn)}
    names = list(ln) + list(rn)
    schema = TableSchema(names, list(left.schema.types) + list(right.schema.types))
    resolve = _resolver(names, qual)
    pred = parse_expr(predicate)
    # hash join on equality conjuncts between the two sides
    eq_l, eq_r = [], []
    for c in _split_and(pred):
        if c.kind == "cmp" and c.args[0] == "=" and c.args[1].kind == "col" and c.args[2].kind == "col":
            i, j = resolve(c.args[1].args[0]), resolve(c.args[2].args[0])
            if i < len(ln) <= j:
                eq_l.append(i)
                eq_r.append(j - len(ln))
            elif j < len(ln) <= i:
                eq_l.append(j)
                eq_r.append(i - len(ln))
    if eq_l:
        res = _join_columnar(left, right, pred, eq_l, eq_r, how, select, schema, qual, resolve)
        if res is not None:
            return res
    if left.num_rows * right.num_rows <= _BLOCKED_JOIN_MAX_PAIRS:
        res = _join_blocked(left, right, pred, how, select, schema, qual, resolve)
        if res is not None:
            return res
    pf = compile_expr(pred, resolve)
    lrows, rrows = left.rows(), right.rows()
    nl, nr = (None,) * len(ln), (None,) * len(rn)
    out = []
    r_matched = [False] * len(rrows)
    if eq_l:
        index = {}
        for j, r in enumerate(rrows):
            index.setdefault(tuple(_key(r[x]) for x in eq_r), []).append(j)
        for l in lrows:
            cands = index.get(tuple(_key(l[x]) for x in eq_l), [])
            hit = False
            for j in cands:
                row = tuple(l) + tuple(rrows[j])
                if pf(row) is True:
                    out.append(row)
                    r_matched[j] = True
                    hit = True
            if not hit and how in ("left", "full"):
                out.append(tuple(l) + nr)
    else:
        for l in lrows:
            hit = False
            for j, r in enumerate(rrows):
                row = tuple(l) + tuple(r)
                if pf(row) is True:
                    out.append(row)
                    r_matched[j] = True
                    hit = True
            if not hit and how in ("left", "full"):
                out.append(tuple(l) + nr)
    if how in ("right", "full"):
        for j, r in enumerate(rrows):
            if not r_matched[j]:
                out.append(nl + tuple(r))
    rows, sch = _select_rows([Row(r) for r in out], schema, select, qual)
    return MTable.from_rows(rows, sch)


# ---------------------------------------------------------------------------------------------------
# columnar equi-join and set operations: joint key codes -> sort / searchsorted on the key columns' device
# ---------------------------------------------------------------------------------------------------
def _null_mask(c) -> "torch.Tensor":
    import torch
    from ....common.strings import StringBlock
    v = c.values
    if isinstance(v, StringBlock):
        return v.null_mask().cpu()
    if isinstance(v, torch.Tensor):
        return c.nulls.cpu() if c.nulls is not None else torch.zeros(int(v.shape[0]), dtype=torch.bool)
    return torch.tensor([x is None for x in v], dtype=torch.bool)


def _joint_codes(lcols, rcols, dev):
    """int64 codes of the key tuples of both sides over one shared dictionary (equal tuples <-> equal codes);
    a row with a NULL in any key gets -1 (left) / -2 (right), so it matches nothing (SQL ``=`` on NULL is not
    TRUE).  None when a key column cannot be factorised columnar."""
    import torch
    from ....common.table import Column
    nl = len(lcols[0]) if lcols else 0
    code = None
    lnull = torch.zeros(nl, dtype=torch.bool)
    rnull = torch.zeros(len(rcols[0]) if rcols else 0, dtype=torch.bool)
    for lc, rc in zip(lcols, rcols):
        lv, rv = lc.values, rc.values
        if isinstance(lv, torch.Tensor) and isinstance(rv, torch.Tensor):
            if lv.dim() != 1 or rv.dim() != 1 or (lv.dtype == torch.bool) != (rv.dtype == torch.bool):
                return None
            if lv.dtype != rv.dtype:       # 1 = 1.0 (the row path compares Python numbers)
                lc = Column(lv.to(torch.float64), lc.nulls)
                rc = Column(rv.to(torch.float64), rc.nulls)
        elif isinstance(lv, torch.Tensor) or isinstance(rv, torch.Tensor):
            return None                    # tensor vs object keys: leave the mixed semantics to the row path
        ci, k = _factorize(Column.concat([lc, rc]))
        if ci is None:
            return None
        ci = ci.to(dev)
        code = ci if code is None else torch.unique(code * k + ci, return_inverse=True)[1]
        lnull |= _null_mask(lc)
        rnull |= _null_mask(rc)
    lk, rk = code[:nl].clone(), code[nl:].clone()
    lk[lnull.to(dev)] = -1
    rk[rnull.to(dev)] = -2
    return lk, rk


def _take_or_null(c, idx, n: int):
    """Rows ``idx`` of column ``c`` (length ``n``); index -1 yields NULL (outer-join padding)."""
    import torch
    from ....common.linalg.block import SparseBlock
    from ....common.strings import StringBlock
    from ....common.table import Column
    neg = idx < 0
    if not bool(neg.any()):
        return c.take(idx)
    v = c.values
    ii = torch.where(neg, torch.full_like(idx, n), idx)          # row n = an appended NULL row
    if isinstance(v, StringBlock):
        return Column(StringBlock.concat([v, StringBlock.from_list([None], device=v.device)]).take(ii.to(v.device)))
    if isinstance(v, torch.Tensor) and v.dim() == 1:
        vals = torch.cat([v, torch.zeros(1, dtype=v.dtype, device=v.device)])[ii.to(v.device)]
        base = c.nulls.to(v.device) if c.nulls is not None else torch.zeros(n, dtype=torch.bool, device=v.device)
        nulls = torch.cat([base, torch.ones(1, dtype=torch.bool, device=v.device)])[ii.to(v.device)]
        return Column(vals, nulls)
    lst = c.to_list() + [None]
    return Column([lst[i] for i in ii.cpu().tolist()])


def _join_columnar(left, right, pred, eq_l, eq_r, how, select, schema, qual, resolve) -> Optional[MTable]:
    """Equi-join without per-row Python: joint key codes, a stable sort of the right side's codes, per left
    row a searchsorted range of matching right rows (repeat_interleave expands the pairs), the residual
    conjuncts evaluated columnar (``vexpr``) on the candidate pairs, outer padding by index -1.  Output row
    order equals the row path's: left rows in order with their matches in right-row order, then (right / full)
    the unmatched right rows in order.  None -> the row path."""
    import torch
    from ....common.table import Column
    from .vexpr import try_evaluate
    nl, nr = left.num_rows, right.num_rows
    dev = next((c.values.device for c in [left.cols[i] for i in eq_l] + [right.cols[j] for j in eq_r]
                if isinstance(c.values, torch.Tensor)), torch.device("cpu"))
    if nl and nr:
        codes = _joint_codes([left.cols[i] for i in eq_l], [right.cols[j] for j in eq_r], dev)
        if codes is None:
            return None
        lk, rk = codes
        order = torch.argsort(rk, stable=True)
        rs = rk[order]
        lo = torch.searchsorted(rs, lk, right=False)
        cnt = torch.searchsorted(rs, lk, right=True) - lo
        cnt = torch.where(lk < 0, torch.zeros_like(cnt), cnt)
        li = torch.repeat_interleave(torch.arange(nl, device=dev), cnt)
        off = torch.cumsum(cnt, 0) - cnt
        ri = order[torch.arange(li.numel(), device=dev) - off[li] + lo[li]]
    else:
        li = torch.zeros(0, dtype=torch.int64, device=dev)
        ri = torch.zeros(0, dtype=torch.int64, device=dev)
    # residual conjuncts (everything but the key equalities): columnar on the candidate pairs
    eqs = set(zip(eq_l, eq_r))
    rest = []
    for c in _split_and(pred):
        if c.kind == "cmp" and c.args[0] == "=" and c.args[1].kind == "col" and c.args[2].kind == "col":
            i, j = resolve(c.args[1].args[0]), resolve(c.args[2].args[0])
            if (i, j - len(left.cols)) in eqs or (j, i - len(left.cols)) in eqs:
                continue
        rest.append(c)
    if rest and li.numel():
        cand = _pair_table(left, right, li, ri, schema, _need(rest, resolve), lambda c, i, n: c.take(i))
        keep = None
        for c in rest:
            r = try_evaluate(c, cand, resolve)
            if r is None or r[0].dtype != torch.bool:
                f = compile_expr(c, resolve)
                m = torch.tensor([f(row) is True for row in cand.rows()], dtype=torch.bool, device=dev)
            else:
                m = (r[0] if r[1] is None else r[0] & ~r[1]).to(dev)
            keep = m if keep is None else keep & m
        li, ri = li[keep], ri[keep]
    return _finish_join(left, right, li, ri, how, select, schema, qual, dev)


def _pair_table(left, right, li, ri, schema, need, take) -> MTable:
    """The (li, ri) pairs as a table of the joined schema; only the columns in ``need`` are gathered (the
    others are inert placeholders nothing reads)."""
    import torch
    from ....common.table import Column
    n = int(li.numel())
    cols = list(left.cols) + list(right.cols)
    nl_cols = len(left.cols)
    out = []
    for i, c in enumerate(cols):
        if i not in need:
            out.append(Column(torch.zeros(n, dtype=torch.bool)))
        elif i < nl_cols:
            out.append(take(c, li, left.num_rows))
        else:
            out.append(take(c, ri, right.num_rows))
    return MTable(schema, out)


def _need(exprs, resolve) -> set:
    return {resolve(nm) for e in exprs for nm in e.columns()}


def _finish_join(left, right, li, ri, how, select, schema, qual, dev) -> MTable:
    """Matched pairs (li, ri) in the row path's order -> outer padding (index -1 = NULL row) -> select."""
    import torch
    nl, nr = left.num_rows, right.num_rows
    if how in ("left", "full"):
        hit = torch.zeros(nl, dtype=torch.bool, device=dev)
        hit[li] = True
        ul = torch.nonzero(~hit).reshape(-1)
        if ul.numel():
            li = torch.cat([li, ul])
            ri = torch.cat([ri, torch.full_like(ul, -1)])
            o = torch.argsort(li, stable=True)            # unmatched left rows at their position
            li, ri = li[o], ri[o]
    if how in ("right", "full"):
        hit = torch.zeros(nr, dtype=torch.bool, device=dev)
        hit[ri[ri >= 0]] = True
        ur = torch.nonzero(~hit).reshape(-1)
        li = torch.cat([li, torch.full_like(ur, -1)])
        ri = torch.cat([ri, ur])
    items = _expand_star(parse_select_list(select), schema)
    need = _need([it.expr for it in items], _resolver(schema.names, qual))
    joined = _pair_table(left, right, li, ri, schema, need, _take_or_null)
    return sql_select(joined, select, qual)


def _join_blocked(left, right, pred, how, select, schema, qual, resolve, pairs: int = 1 << 21) -> Optional[MTable]:
    """Joins without usable equality keys (theta joins such as ``a.x < b.y``, or key columns that do not
    factorise): the left x right pairs in blocks of whole left rows, the predicate evaluated columnar (``vexpr``)
    on each block -- the same O(nl * nr) comparisons as the nested loop, without per-pair Python.  Pair order is
    the nested loop's.  None when the predicate has no columnar form (the row path then runs it)."""
    import torch
    from .vexpr import try_evaluate
    nl, nr = left.num_rows, right.num_rows
    dev = next((c.values.device for c in list(left.cols) + list(right.cols) if isinstance(c.values, torch.Tensor)),
               torch.device("cpu"))
    lis, ris = [], []
    if nl and nr:
        step = max(1, pairs // nr)
        rr = torch.arange(nr, device=dev)
        for a in range(0, nl, step):
            b = min(nl, a + step)
            li = torch.arange(a, b, device=dev).repeat_interleave(nr)
            ri = rr.repeat(b - a)
            cand = _pair_table(left, right, li, ri, schema, _need([pred], resolve), lambda c, i, n: c.take(i))
            r = try_evaluate(pred, cand, resolve)
            if r is None or r[0].dtype != torch.bool:
                return None
            m = (r[0] if r[1] is None else r[0] & ~r[1]).to(dev)
            lis.append(li[m])
            ris.append(ri[m])
    li = torch.cat(lis) if lis else torch.zeros(0, dtype=torch.int64, device=dev)
    ri = torch.cat(ris) if ris else torch.zeros(0, dtype=torch.int64, device=dev)
    return _finish_join(left, right, li, ri, how, select, schema, qual, dev)


def _set_codes(a: MTable, b: MTable):
    """Row codes of ``a`` and ``b`` over one dictionary (NULLs equal each other, as set operations treat them);
    None -> the row path."""
    import torch
    if a.num_rows == 0 or b.num_rows == 0:
        return None
    both = MTable.concat([a, MTable(a.schema, b.cols, a.replicated)])
    dev = next((c.values.device for c in both.cols if isinstance(c.values, torch.Tensor)), torch.device("cpu"))
    code = _row_codes(both, range(len(both.cols)), dev)
    if code is None:
        return None
    return code[:a.num_rows], code[a.num_rows:], int(code.max()) + 1


def _occurrence_rank(code):
    """Per row: how many earlier rows carry the same code (stable)."""
    import torch
    o = torch.argsort(code, stable=True)
    sc = code[o]
    pos = torch.arange(code.numel(), device=code.device)
    start = torch.searchsorted(sc, sc, right=False)
    rank = torch.empty_like(o)
    rank[o] = pos - start
    return rank


def _set_op_columnar(a: MTable, b: MTable, all_: bool, keep_common: bool) -> Optional[MTable]:
    import torch
    sc = _set_codes(a, b)
    if sc is None:
        return None
    ca, cb, G = sc
    nb = torch.bincount(cb, minlength=G)
    r = _occurrence_rank(ca)
    if all_:
        keep = r < nb[ca] if keep_common else r >= nb[ca]
    else:
        keep = (r == 0) & ((nb[ca] > 0) if keep_common else (nb[ca] == 0))
    return a.take(torch.nonzero(keep).reshape(-1))


def sql_union(a: MTable, b: MTable, all_: bool) -> MTable:
    b2 = MTable(a.schema, b.cols, a.replicated)
    u = MTable.concat([a, b2])
    return u if all_ else sql_distinct(u)


def sql_intersect(a: MTable, b: MTable, all_: bool) -> MTable:
    res = _set_op_columnar(a, b, all_, True)
    if res is not None:
        return res
    cb = Counter(tuple(_key(v) for v in r) for r in b.rows())
    keep, seen = [], set()
    for i, r in enumerate(a.rows()):
        k = tuple(_key(v) for v in r)
        if cb.get(k, 0) > 0:
            if all_:
                cb[k] -= 1
                keep.append(i)
            elif k not in seen:
                seen.add(k)
                keep.append(i)
    return a.take(keep)


def sql_minus(a: MTable, b: MTable, all_: bool) -> MTable:
    res = _set_op_columnar(a, b, all_, False)
    if res is not None:
        return res
    cb = Counter(tuple(_key(v) for v in r) for r in b.rows())
    keep, seen = [], set()
    for i, r in enumerate(a.rows()):
        k = tuple(_key(v) for v in r)
        if all_:
            if cb.get(k, 0) > 0:
                cb[k] -= 1
            else:
                keep.append(i)
        elif k not in cb and k not in seen:
            seen.add(k)
            keep.append(i)
    return a.take(keep)


# ---------------------------------------------------------------------------------------------------
# distributed plan helpers (operator/batch/sql.py): which columns co-partition an operator's inputs
# ---------------------------------------------------------------------------------------------------
def join_keys(left: TableSchema, right: TableSchema, predicate: str) -> Tuple[List[int], List[int]]:
    """Column indices of the equality conjuncts ``a.x = b.y`` of a join predicate (empty: not an equi-join)."""
    ln, rn = left.names, right.names
    qual = {"a": (0, ln), "b": (len(ln), rn)}
    resolve = _resolver(list(ln) + list(rn), qual)
    eq_l, eq_r = [], []
    for c in _split_and(parse_expr(predicate)):
        if c.kind == "cmp" and c.args[0] == "=" and c.args[1].kind == "col" and c.args[2].kind == "col":
            i, j = resolve(c.args[1].args[0]), resolve(c.args[2].args[0])
            if i < len(ln) <= j:
                eq_l.append(i)
                eq_r.append(j - len(ln))
            elif j < len(ln) <= i:
                eq_l.append(j)
                eq_r.append(i - len(ln))
    return eq_l, eq_r


def group_key_cols(schema: TableSchema, by: str) -> Optional[List[int]]:
    """Indices of the group-by items when every item is a plain column reference, else None."""
    resolve = _resolver(schema.names)
    out = []
    for p in split_top_level(by):
        e = parse_expr(p)
        if e.kind != "col":
            return None
        out.append(resolve(e.args[0]))
    return out


def order_key_fn(mt: MTable, clause: str, order: str = "asc"):
    """Row -> sort key of ``sql_order_by`` (nulls first ascending / last descending, per-key direction), as a
    ``functools.cmp_to_key`` object usable for splitters and bisection."""
    import functools
    keys = []
    for part in split_top_level(clause):
        toks = part.split()
        asc = order.lower() != "desc"
        if len(toks) > 1 and toks[-1].lower() in ("asc", "desc"):
            asc = toks[-1].lower() == "asc"
            part = " ".join(toks[:-1])
        keys.append((compile_expr(parse_expr(part), _resolver(mt.schema.names)), asc))

    def cmp(x, y):
        for (f, asc), a, b in zip(keys, x, y):
            ka = (a is not None, a if a is not None else 0)
            kb = (b is not None, b if b is not None else 0)
            if ka != kb:
                r = -1 if ka < kb else 1
                return r if asc else -r
        return 0

    K = functools.cmp_to_key(cmp)
    return lambda row: K(tuple(f(row) for f, _ in keys))

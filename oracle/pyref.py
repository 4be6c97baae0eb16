"""Pure-Python literal restatement of circom's R1CS simplification (--O1 / --O2 / --O2round).

TEST INFRASTRUCTURE -- ORACLE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use anything under oracle/.  This module is never on the product path.

It restates, function by function, the reference at /root/reference (circom 2.2.2 / circom_cvm):

  constraint_list/src/constraint_simplification.rs   (build_clusters, rebuild_witness,
      eq_cluster_simplification, eq_simplification, constant_eq_simplification,
      linear_simplification, build_non_linear_signal_map, apply_substitution_to_map,
      build_relevant_set, remove_not_relevant, simplification)
  constraint_list/src/non_linear_utils.rs             (obtain_and_simplify_non_linear)
  circom_algebra/src/simplification_utils.rs          (full_simplification and helpers)
  circom_algebra/src/algebra.rs                       (ArithmeticExpression / Substitution /
      Constraint operations, raw_substitution, fix_raw_constraint, ...)
  circom_algebra/src/modular_arithmetic.rs            (add, mul, sub, div, multi_inv)
  dag/src/map_to_constraint_list.rs:12-44             (classification of the --O0 rows)
  constraint_list/src/r1cs_porting.rs + constraint_writers/src/r1cs_writer.rs (.r1cs bytes)
  constraint_list/src/sym_porting.rs + constraint_writers/src/sym_writer.rs   (.sym text)

Rust HashMap<usize, BigInt> maps are Python dicts (explicit keys, zero values allowed, exactly like
the reference's maps).  Wherever the reference iterates a HashMap/HashSet in an order-sensitive
place, this restatement iterates in ASCENDING key order and collects thread-pool results in
CLUSTER-INDEX order: the canonical legal execution of SURVEY.md section 8(a) row A22.

It is deliberately slow and literal; use it on small systems only.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field as dc_field
from typing import Dict, List, Optional, Tuple

# program_structure/src/utils/constants.rs:3-13
PRIMES = {
    "bn128": 21888242871839275222246405745257275088548364400416034343698204186575808495617,
    "bls12381": 52435875175126190479447740508185965837690552500527637822603658699938581184513,
    "goldilocks": 18446744069414584321,
    "grumpkin": 21888242871839275222246405745257275088696311157297823662689037894645226208583,
    "pallas": 28948022309329048855892746252171976963363056481941560715954676764349967630337,
    "vesta": 28948022309329048855892746252171976963363056481941647379679742748393362948097,
    "secq256r1": 115792089210356248762697446949407573530086143415290314195533631308867097853951,
    "bls12377": 8444461749428370424248824938781546531375899335154063827935233455917409239041,
}

Map = Dict[int, int]          # HashMap<usize, BigInt>
CONST = 0                      # ArithmeticExpression::constant_coefficient() == usize::default()


# ----------------------------------------------------------------- modular_arithmetic.rs:9-91
def modulus(a: int, b: int) -> int:
    return ((a % b) + b) % b


def m_add(a, b, p):
    return modulus(a + b, p)


def m_mul(a, b, p):
    return modulus(a * b, p)


def m_sub(a, b, p):
    return modulus(a - b, p)


def m_div(a, b, p):
    inv = pow(b, -1, p)          # mod_inverse; raises ValueError on 0 (DivisionByZero)
    return m_mul(a, inv, p)


def multi_inv(values: List[int], p: int) -> List[int]:
    """modular_arithmetic.rs:71-91 (Montgomery batch inversion)."""
    partials = [1]
    for v in values:
        partials.append(m_mul(partials[-1], v, p))
    inverse = m_div(1, partials[-1], p)
    out = [0] * len(partials)
    i = len(values)
    while i > 0:
        out[i - 1] = m_mul(partials[i - 1], inverse, p)
        inverse = m_mul(inverse, values[i - 1], p)
        i -= 1
    return out


# ----------------------------------------------------------------- algebra.rs: expressions
class AE:
    """ArithmeticExpression<usize> (algebra.rs:9-34).  kind in {Number, Signal, Linear}."""
    __slots__ = ("kind", "value", "symbol", "coefs")

    def __init__(self, kind, value=None, symbol=None, coefs=None):
        self.kind, self.value, self.symbol, self.coefs = kind, value, symbol, coefs

    @staticmethod
    def number(v):
        return AE("Number", value=v)

    @staticmethod
    def signal(s):
        return AE("Signal", symbol=s)

    @staticmethod
    def linear(m):
        return AE("Linear", coefs=m)

    def clone(self):
        return AE(self.kind, self.value, self.symbol, dict(self.coefs) if self.coefs is not None else None)


def init_map(m: Map) -> None:
    """initialize_hashmap_for_expression (algebra.rs:158-163)."""
    if CONST not in m:
        m[CONST] = 0


def add_constant_to_coefficients(value, m: Map, p):
    m[CONST] = m_add(m[CONST], value, p)


def add_symbol_to_coefficients(sym, coef, m: Map, p):
    if sym not in m:
        m[sym] = 0
    m[sym] = m_add(m[sym], coef, p)


def add_coefficients_to_coefficients(m0: Map, m1: Map, p):
    for k in sorted(m0):
        add_symbol_to_coefficients(k, m0[k], m1, p)


def multiply_coefficients_by_constant(c, m: Map, p):
    for k in list(m.keys()):
        m[k] = m_mul(m[k], c, p)


def divide_coefficients_by_constant(c, m: Map, p):
    inv = m_div(1, c, p)
    multiply_coefficients_by_constant(inv, m, p)


def ae_add(l: AE, r: AE, p) -> AE:
    """algebra.rs:247-347 (the Number/Signal/Linear cases used on this path)."""
    K = (l.kind, r.kind)
    if K == ("Number", "Number"):
        return AE.number(m_add(l.value, r.value, p))
    if K in (("Number", "Signal"), ("Signal", "Number")):
        n, s = (l, r) if l.kind == "Number" else (r, l)
        m: Map = {}
        init_map(m)
        add_constant_to_coefficients(n.value, m, p)
        add_symbol_to_coefficients(s.symbol, 1, m, p)
        return AE.linear(m)
    if K in (("Number", "Linear"), ("Linear", "Number")):
        n, li = (l, r) if l.kind == "Number" else (r, l)
        m = dict(li.coefs)
        add_constant_to_coefficients(n.value, m, p)
        return AE.linear(m)
    if K == ("Signal", "Signal"):
        m = {}
        init_map(m)
        add_symbol_to_coefficients(l.symbol, 1, m, p)
        add_symbol_to_coefficients(r.symbol, 1, m, p)
        return AE.linear(m)
    if K in (("Signal", "Linear"), ("Linear", "Signal")):
        s, li = (l, r) if l.kind == "Signal" else (r, l)
        m = dict(li.coefs)
        add_symbol_to_coefficients(s.symbol, 1, m, p)
        return AE.linear(m)
    if K == ("Linear", "Linear"):
        m = dict(r.coefs)
        add_coefficients_to_coefficients(l.coefs, m, p)
        return AE.linear(m)
    raise NotImplementedError(K)


def ae_mul(l: AE, r: AE, p) -> AE:
    """algebra.rs:349-440 (the linear-result cases used on this path)."""
    K = (l.kind, r.kind)
    if K == ("Number", "Number"):
        return AE.number(m_mul(l.value, r.value, p))
    if K in (("Number", "Signal"), ("Signal", "Number")):
        n, s = (l, r) if l.kind == "Number" else (r, l)
        m: Map = {}
        init_map(m)
        add_symbol_to_coefficients(s.symbol, n.value, m, p)
        return AE.linear(m)
    if K in (("Number", "Linear"), ("Linear", "Number")):
        n, li = (l, r) if l.kind == "Number" else (r, l)
        m = dict(li.coefs)
        multiply_coefficients_by_constant(n.value, m, p)
        return AE.linear(m)
    raise NotImplementedError(K)


def ae_sub(l: AE, r: AE, p) -> AE:
    """algebra.rs:441-450."""
    return ae_add(l, ae_mul(AE.number(-1), r, p), p)


def hashmap_into_arith(m: Map) -> AE:
    """algebra.rs:804-825."""
    m = dict(m)
    if len(m) == 1 and CONST in m:
        return AE.number(m.pop(CONST))
    if len(m) == 1:
        (sym, val), = m.items()
        if val == 1:
            return AE.signal(sym)
        init_map(m)
        return AE.linear(m)
    init_map(m)
    return AE.linear(m)


@dataclass
class Sub:
    """Substitution<usize> (algebra.rs:835-841): from := to."""
    frm: int
    to: Map


def sub_new(frm: int, expr: AE) -> Optional[Sub]:
    """Substitution::new (algebra.rs:844-862)."""
    if expr.kind == "Number":
        return Sub(frm, {CONST: expr.value})
    if expr.kind == "Signal":
        return Sub(frm, {expr.symbol: 1})
    if expr.kind == "Linear" and frm not in expr.coefs:
        return Sub(frm, expr.coefs)
    return None


def sub_decompose(s: Sub) -> Tuple[int, AE]:
    """Substitution::decompose (algebra.rs:906-928)."""
    to = dict(s.to)
    if len(to) == 1 and CONST in to:
        return s.frm, AE.number(to.pop(CONST))
    if len(to) == 1:
        (sym, val), = to.items()
        if val == 1:
            return s.frm, AE.signal(sym)
        init_map(to)
        return s.frm, AE.linear(to)
    init_map(to)
    return s.frm, AE.linear(to)


def raw_substitution(change: Map, sub: Sub, p) -> None:
    """algebra.rs:1279-1294 (no zero pruning)."""
    init_map(change)
    if sub.frm in change:
        val = change.pop(sub.frm)
        coefs = dict(sub.to)
        init_map(coefs)
        multiply_coefficients_by_constant(val, coefs, p)
        add_coefficients_to_coefficients(coefs, change, p)


def remove_zero(m: Map) -> Map:
    """remove_zero_value_coefficients (algebra.rs:1296-1307)."""
    return {k: v for k, v in m.items() if v != 0}


@dataclass
class Con:
    """Constraint<usize>: A*B - C = 0 (algebra.rs:997-1009)."""
    a: Map
    b: Map
    c: Map

    def clone(self):
        return Con(dict(self.a), dict(self.b), dict(self.c))


def con_empty() -> Con:
    return Con({}, {}, {})


def is_empty(c: Con) -> bool:
    return not c.a and not c.b and not c.c


def is_linear(c: Con) -> bool:
    return not c.a and not c.b


def take_cloned_signals(c: Con) -> List[int]:
    """algebra.rs:1078-1091 (a HashSet; returned ascending = canonical iteration order)."""
    s = set(c.a) | set(c.b) | set(c.c)
    s.discard(CONST)
    return sorted(s)


def apply_substitution(c: Con, sub: Sub, p) -> None:
    """Constraint::apply_substitution (algebra.rs:1138-1147)."""
    raw_substitution(c.a, sub, p)
    raw_substitution(c.b, sub, p)
    raw_substitution(c.c, sub, p)


def is_constant_expression(m: Map) -> bool:
    return CONST in m and len(m) == 1


def constant_linear_linear_reduction(a: Map, b: Map, c: Map, p) -> Map:
    """algebra.rs:1326-1344; returns the new c (a and b are cleared in place)."""
    init_map(c)
    init_map(b)
    constant = a.pop(CONST)
    multiply_coefficients_by_constant(constant, b, p)
    multiply_coefficients_by_constant(-1, b, p)
    add_coefficients_to_coefficients(b, c, p)
    c = remove_zero(c)
    a.clear()
    b.clear()
    return c


def fix_constraint(con: Con, p) -> None:
    """fix_raw_constraint (algebra.rs:1309-1324)."""
    con.a = remove_zero(con.a)
    con.b = remove_zero(con.b)
    con.c = remove_zero(con.c)
    if not con.a or not con.b:
        con.a.clear()
        con.b.clear()
    elif is_constant_expression(con.a):
        con.c = constant_linear_linear_reduction(con.a, con.b, con.c, p)
    elif is_constant_expression(con.b):
        con.c = constant_linear_linear_reduction(con.b, con.a, con.c, p)


def clear_signal(symbols: Map, key: int, p) -> Map:
    """algebra.rs:1108-1124."""
    symbols = dict(symbols)
    key_value = symbols.pop(key)
    assert key_value != 0
    vtr = m_mul(key_value, -1, p)
    init_map(symbols)
    divide_coefficients_by_constant(vtr, symbols, p)
    return remove_zero(symbols)


def clear_signal_not_normalized(symbols: Map, key: int, p) -> Tuple[int, Map]:
    """algebra.rs:1126-1136."""
    symbols = dict(symbols)
    key_value = symbols.pop(key)
    assert key_value != 0
    vtr = m_mul(key_value, -1, p)
    init_map(symbols)
    return vtr, symbols


def transform_expression_to_constraint_form(e: AE, p) -> Con:
    """algebra.rs:113-145 (C := -expr)."""
    a: Map = {}
    b: Map = {}
    c: Map = {}
    init_map(a)
    init_map(b)
    init_map(c)
    if e.kind == "Number":
        c[CONST] = e.value
    elif e.kind == "Signal":
        c[e.symbol] = 1
    elif e.kind == "Linear":
        c = dict(e.coefs)
    else:
        raise NotImplementedError(e.kind)
    multiply_coefficients_by_constant(-1, c, p)
    return Con(a, b, c)


def remove_zero_con(c: Con) -> None:
    c.a = remove_zero(c.a)
    c.b = remove_zero(c.b)
    c.c = remove_zero(c.c)


def is_constant_equality(con: Con) -> bool:
    """signal_equals_constant (algebra.rs:1362-1372)."""
    c = con.c
    return (not con.a and not con.b and
            ((CONST in c and len(c) == 2) or (CONST not in c and len(c) == 1)))


def is_equality(con: Con, p) -> bool:
    """signal_equals_signal (algebra.rs:1346-1360)."""
    c = con.c
    if not con.a and not con.b and CONST not in c and len(c) == 2:
        k0, k1 = list(c.keys())
        return m_mul(-1, c[k1], p) == c[k0]
    return False


# ----------------------------------------------------------------- constraint_simplification.rs
def build_clusters(linear: List[Con], no_vars: int) -> List[List[Con]]:
    """constraint_simplification.rs:45-99."""
    arena: List[Optional[List[Con]]] = []
    c2c: List[int] = []
    sig2cl: Dict[int, int] = {}

    def find(org):
        cur = org
        while cur != c2c[cur]:
            cur = c2c[cur]
        return cur

    def merge(src, dest):
        cd, cs = find(dest), find(src)
        c0 = arena[cd] or []
        arena[cd] = None
        c1 = arena[cs] or []
        arena[cs] = None
        arena[cd] = c0 + c1
        c2c[cs] = cd

    for con in linear:
        if not is_empty(con):
            signals = take_cloned_signals(con)
            dest = len(arena)
            arena.append([con])
            c2c.append(dest)
            for s in signals:
                prev = sig2cl.get(s)
                sig2cl[s] = dest
                if prev is not None:
                    merge(prev, dest)
    return [cl for cl in arena if cl is not None and len(cl) != 0]


def rebuild_witness(max_signal, deleted: set, forbidden: set, nl_map: dict, remove_unused=True):
    """constraint_simplification.rs:101-124."""
    out = {}
    free: List[int] = []
    head = 0
    for s in range(max_signal):
        if s in deleted:
            free.append(s)
        elif remove_unused and s not in forbidden and s not in nl_map:
            deleted.add(s)
            free.append(s)
        elif head < len(free):
            out[s] = free[head]
            head += 1
            free.append(s)
        else:
            out[s] = s
    return out


def eq_cluster_simplification(cluster: List[Con], forbidden: set, p):
    """constraint_simplification.rs:126-196."""
    if len(cluster) == 1:
        subs, cons = [], []
        con = cluster[-1]
        s0, s1 = take_cloned_signals(con)[:2]
        if s0 in forbidden and s1 in forbidden:
            cons.append(con)
        elif s0 in forbidden:
            subs.append(sub_new(s1, AE.signal(s0)))
        elif s1 in forbidden:
            subs.append(sub_new(s0, AE.signal(s1)))
        else:
            l, r = (s0, s1) if s0 > s1 else (s1, s0)
            subs.append(sub_new(l, AE.signal(r)))
        return subs, cons
    cons, subs = [], []
    remains, remove = set(), set()
    min_remains = min_remove = None
    for c in cluster:
        for s in take_cloned_signals(c):
            if s in forbidden:
                remains.add(s)
                min_remains = s if min_remains is None else min(min_remains, s)
            else:
                min_remove = s if min_remove is None else min(min_remove, s)
                remove.add(s)
    if min_remains is not None:
        remains.discard(min_remains)
        rh = min_remains
    else:
        rh = min_remove
        remove.discard(rh)
    for s in sorted(remains):
        expr = ae_sub(AE.signal(s), AE.signal(rh), p)
        cons.append(transform_expression_to_constraint_form(expr, p))
    for s in sorted(remove):
        subs.append(sub_new(s, AE.signal(rh)))
    return subs, cons


def eq_simplification(equalities, forbidden, no_vars, p, log):
    """constraint_simplification.rs:198-251 (ThreadPool results collected by cluster id)."""
    clusters = build_clusters(equalities, no_vars)
    aux = [[] for _ in clusters]
    subs: List[Sub] = []
    deferred = []
    for cid, cl in enumerate(clusters):
        if len(cl) == 1:
            s, c = eq_cluster_simplification(cl, forbidden, p)
            aux[cid] = c
            subs += s
        else:
            deferred.append(cid)
    for cid in deferred:
        s, c = eq_cluster_simplification(clusters[cid], forbidden, p)
        aux[cid] = c
        subs += s
    cons = [c for cl in aux for c in cl]
    if log is not None:
        log.extend(subs)
    return subs, cons


def constant_eq_simplification(c_eq, forbidden, p, log):
    """constraint_simplification.rs:253-273."""
    cons, subs = [], []
    for con in c_eq:
        signal = take_cloned_signals(con)[-1]
        if signal in forbidden:
            cons.append(con)
        else:
            subs.append(Sub(signal, clear_signal(con.c, signal, p)))
    if log is not None:
        log.extend(subs)
    return subs, cons


# ----------------------------------------------------------------- simplification_utils.rs
def take_signal_3(forbidden, work: Con):
    """simplification_utils.rs:368-377."""
    ret = None
    for k in sorted(work.c):
        if k not in forbidden:
            ret = k if ret is None else max(ret, k)
    return ret


def take_signal_4(forbidden, deleted, occ, work: Con):
    """simplification_utils.rs:379-411 (HashMap order := ascending)."""
    ret = None
    occ_ret = None
    for k in sorted(work.c):
        if k not in forbidden:
            if k in deleted:
                ret = k
                break
            n = occ[k]
            if occ_ret is None:
                ret, occ_ret = k, n
            elif n < occ_ret:
                ret, occ_ret = k, n
            elif n == occ_ret and ret < k:
                ret = k
    return ret


def merge_conflict(coef, sub_to, in_coef, in_to, p) -> Con:
    """treat_constraint_3/4 conflict merge (simplification_utils.rs:283-292, 338-347)."""
    right = sub_decompose(Sub(0, in_to))[1]
    left = sub_decompose(Sub(0, sub_to))[1]
    new_left = ae_mul(AE.number(in_coef), left, p)
    new_right = ae_mul(AE.number(coef), right, p)
    merge = ae_sub(new_left, new_right, p)
    work = transform_expression_to_constraint_form(merge, p)
    remove_zero_con(work)
    return work


def substitution_process_3(forbidden, constraints: List[Con], holder: dict, p) -> List[Con]:
    """simplification_utils.rs:143-154 + treat_constraint_3 (:259-294)."""
    lconst = []
    deleted = set()
    cons = list(constraints)
    while cons:
        work = cons.pop()
        while True:
            if is_empty(work):
                break
            out = take_signal_3(forbidden, work)
            if out is None:
                lconst.append(work)
                break
            deleted.add(out)
            coef, to = clear_signal_not_normalized(work.c, out, p)
            if out not in holder:
                holder[out] = (coef, to)
                break
            in_coef, in_to = holder[out]
            work = merge_conflict(coef, to, in_coef, in_to, p)
    return lconst


def substitution_process_4(forbidden, constraints: List[Con], holder: dict, p):
    """simplification_utils.rs:156-185 + SignalsInformation (:60-113) + treat_*_4 (:296-349)."""
    lconst = []
    deleted = set()
    order: List[int] = []           # order_signals: newest first
    vec = [c.clone() for c in constraints]
    occ: Dict[int, int] = {}
    rep: Dict[int, int] = {}
    for pos, c in enumerate(vec):
        for k in c.c:
            if k not in forbidden:
                if k in occ:
                    occ[k] += 1
                else:
                    occ[k] = 1
                    rep[k] = pos
    uniques = sorted((k, rep[k]) for k, n in occ.items() if n == 1)

    def remove_constraint(c: Con):
        for k in c.c:
            if k not in forbidden and k in occ:
                occ[k] -= 1

    def delete(k):
        deleted.add(k)
        order.insert(0, k)

    for signal, index in uniques:
        if not is_empty(vec[index]):
            actual = vec[index]
            vec[index] = con_empty()
            remove_constraint(actual)
            coef, to = clear_signal_not_normalized(actual.c, signal, p)
            holder[signal] = (coef, to)
            occ.pop(signal, None)
            delete(signal)
    while vec:
        work = vec.pop()
        remove_constraint(work)
        while True:
            if is_empty(work):
                break
            out = take_signal_4(forbidden, deleted, occ, work)
            if out is None:
                lconst.append(work)
                break
            coef, to = clear_signal_not_normalized(work.c, out, p)
            if out not in holder:
                delete(out)
                occ.pop(out, None)
                holder[out] = (coef, to)
                break
            in_coef, in_to = holder[out]
            work = merge_conflict(coef, to, in_coef, in_to, p)
    return lconst, order


def normalize_substitutions(holder: dict, p) -> Dict[int, Sub]:
    """simplification_utils.rs:414-437 (BTreeMap: ascending signal)."""
    keys = sorted(holder)
    inverses = multi_inv([holder[k][0] for k in keys], p)
    tree = {}
    for i, s in enumerate(keys):
        arith = hashmap_into_arith(holder[s][1])
        mult = ae_mul(arith, AE.number(inverses[i]), p)
        tree[s] = sub_new(s, mult)
    return tree


def _apply_sub_to_sub(src: Sub, change: Sub, p):
    """Substitution::apply_substitution (algebra.rs:890-892)."""
    raw_substitution(src.to, change, p)


def create_nonoverlapping_substitutions(possible: Dict[int, Sub], p) -> Dict[int, Sub]:
    """simplification_utils.rs:451-463 (BTreeMap ascending)."""
    no_overlap: Dict[int, Sub] = {}
    for s in sorted(possible):
        sub = possible[s]
        to_apply = [no_overlap[k] for k in sorted(sub.to) if k in no_overlap]
        for t in to_apply:
            _apply_sub_to_sub(sub, t, p)
        no_overlap[s] = sub
    return no_overlap


def create_nonoverlapping_substitutions_4(possible: Dict[int, Sub], order, p) -> Dict[int, Sub]:
    """simplification_utils.rs:465-479 (deletion order, newest first)."""
    no_overlap: Dict[int, Sub] = {}
    possible = dict(possible)
    for s in order:
        sub = possible.pop(s)
        to_apply = [no_overlap[k] for k in sorted(sub.to) if k in no_overlap]
        for t in to_apply:
            _apply_sub_to_sub(sub, t, p)
        no_overlap[s] = sub
    return no_overlap


def full_simplification(cluster: List[Con], forbidden, p, use_old_heuristics=False):
    """simplification_utils.rs:543-581.  Result substitutions in ascending `from` (canonical)."""
    n = len(cluster)
    holder: dict = {}
    if 350 <= n < 1000000 and not use_old_heuristics:
        lconst, order = substitution_process_4(forbidden, cluster, holder, p)
        norm = normalize_substitutions(holder, p)
        non_overlap = create_nonoverlapping_substitutions_4(norm, order, p)
    else:
        lconst = substitution_process_3(forbidden, cluster, holder, p)
        norm = normalize_substitutions(holder, p)
        non_overlap = create_nonoverlapping_substitutions(norm, p)
    subs = [non_overlap[s] for s in sorted(non_overlap)]
    return lconst, subs


def linear_simplification(log, linear, forbidden, no_labels, p, use_old_heuristics):
    """constraint_simplification.rs:275-325 (results collected in cluster-index order)."""
    cons, subs = [], []
    for cl in build_clusters(linear, no_labels):
        lc, sb = full_simplification(cl, forbidden, p, use_old_heuristics)
        if log is not None:
            log.extend(sb)
        cons += lc
        subs += sb
    return subs, cons


def fast_encoded_constraint_substitution(c: Con, enc: Dict[int, AE], p) -> bool:
    """simplification_utils.rs:496-507."""
    applied = False
    for s in take_cloned_signals(c):
        if s in enc:
            apply_substitution(c, sub_new(s, enc[s].clone()), p)
            applied = True
    return applied


def build_encoded_fast_substitutions(subs: List[Sub]) -> Dict[int, AE]:
    """simplification_utils.rs:520-527."""
    enc = {}
    for s in subs:
        frm, to = sub_decompose(Sub(s.frm, dict(s.to)))
        enc[frm] = to
    return enc


def build_non_linear_signal_map(storage: List[Con]) -> Dict[int, List[int]]:
    """constraint_simplification.rs:327-343."""
    m: Dict[int, List[int]] = {}
    for cid, c in enumerate(storage):
        for s in take_cloned_signals(c):
            m.setdefault(s, []).append(cid)
    return m


def apply_substitution_to_map(storage: List[Con], m, subs: List[Sub], p) -> List[Con]:
    """constraint_simplification.rs:345-396."""
    linear_id = []
    for sub in subs:
        if sub.frm in m:
            c_ids = list(m[sub.frm])
            signals = sorted(sub.to)
            for cid in c_ids:
                con = storage[cid].clone()
                apply_substitution(con, sub, p)
                fix_constraint(con, p)
                if is_linear(con):
                    linear_id.append(cid)
                storage[cid] = con
                for s in signals:
                    m.setdefault(s, []).append(cid)
    linear = []
    for cid in linear_id:
        linear.append(storage[cid].clone())
        storage[cid] = con_empty()
    return linear


# ----------------------------------------------------------------- the path (CS-2)
@dataclass
class Flags:
    """SimplificationFlags (dag/src/lib.rs:546-554) as consumed by the Simplifier."""
    flag_s: bool = False                     # --O1  (apply_linear = !flag_s)
    no_rounds: int = (1 << 64) - 1           # usize::MAX for --O2; N for --O2round N
    use_old_heuristics: bool = False


@dataclass
class System:
    """What simplification() consumes, reconstructed losslessly from an --O0 export (CS-4)."""
    p: int
    max_signal: int
    n_pub_out: int
    n_pub_in: int
    n_priv_in: int
    forbidden: set
    rows: List[Con]                          # --O0 rows in DFS order
    # custom gates of the --O0 export, or None: (section 4 bytes, [(gate index, [signals])]);
    # the O2 writer re-emits them (constraint_list/src/r1cs_porting.rs:54-121)
    gates: Optional[Tuple[bytes, List[Tuple[int, List[int]]]]] = None


@dataclass
class Result:
    constraints: List[Con]                   # storage order, ORIGINAL signal ids
    signal_map: Dict[int, int]               # label -> wire
    no_private_inputs_witness: int
    log: List[Sub] = dc_field(default_factory=list)


def classify(sys_: System):
    """dag/src/map_to_constraint_list.rs:12-44 + map_node_to_encoding (:71-104)."""
    cons_eq, eq, lin, nonlin = [], [], [], []
    for r in sys_.rows:
        if is_constant_equality(r):
            cons_eq.append(r.clone())
        elif is_equality(r, sys_.p):
            eq.append(r.clone())
        elif is_linear(r):
            lin.append(r.clone())
        if not is_linear(r):
            nonlin.append(r.clone())
    return cons_eq, eq, lin, nonlin


def simplification(sys_: System, flags: Flags, want_log=False) -> Result:
    """constraint_simplification.rs:442-730."""
    p = sys_.p
    log = [] if want_log else None
    apply_linear = not flags.flag_s
    forbidden = set(sys_.forbidden)
    no_labels = sys_.max_signal
    cons_equalities, equalities, linear, non_linear = classify(sys_)
    deleted = set()
    lconst: List[Con] = []
    no_rounds = flags.no_rounds

    def relevant_set(renames, deletes):
        rel = set()
        for c in non_linear:
            for s in take_cloned_signals(c):
                e = renames.get(s)
                s2 = e.symbol if (e is not None and e.kind == "Signal") else s
                if s2 not in deletes:
                    rel.add(s2)
        return rel

    relevant = relevant_set({}, {})

    subs, cons = eq_simplification(equalities, forbidden, no_labels, p, log)
    lconst += cons
    single = build_encoded_fast_substitutions(subs)
    for c in linear:
        if fast_encoded_constraint_substitution(c, single, p):
            fix_constraint(c, p)
    for c in cons_equalities:
        if fast_encoded_constraint_substitution(c, single, p):
            fix_constraint(c, p)
    deleted |= set(single)
    single = {k: v for k, v in single.items() if k in relevant}

    subs, cons = constant_eq_simplification(cons_equalities, forbidden, p, log)
    lconst += cons
    const_subs = build_encoded_fast_substitutions(subs)
    for c in linear:
        if fast_encoded_constraint_substitution(c, const_subs, p):
            fix_constraint(c, p)
    deleted |= set(const_subs)

    relevant = relevant_set(single, const_subs)

    if apply_linear:
        subs, cons = linear_simplification(log, linear, forbidden, no_labels, p,
                                           flags.use_old_heuristics)
        only_relevant = []
        for s in subs:
            deleted.add(s.frm)
            if s.frm in relevant:
                only_relevant.append(s)
        lin_subs = build_encoded_fast_substitutions(only_relevant)
        lconst += cons
        for c in lconst:
            if fast_encoded_constraint_substitution(c, lin_subs, p):
                fix_constraint(c, p)
    else:
        lconst += linear
        lin_subs = {}

    frames = [single, const_subs, lin_subs]
    storage: List[Con] = []
    with_linear: List[Con] = []
    for c0 in non_linear:
        c = c0.clone()
        for fr in frames:
            fast_encoded_constraint_substitution(c, fr, p)
        fix_constraint(c, p)
        if is_linear(c):
            with_linear.append(c)
        else:
            storage.append(c)
    if no_rounds > 0:
        no_rounds -= 1

    linear = with_linear
    apply_round = apply_linear and no_rounds > 0 and len(linear) > 0
    nl_map = build_non_linear_signal_map(storage)
    while apply_round:
        subs, constants = linear_simplification(log, linear, forbidden, no_labels, p,
                                                flags.use_old_heuristics)
        for s in subs:
            deleted.add(s.frm)
        lconst += constants
        for c in lconst:
            for s in subs:
                apply_substitution(c, s, p)
            fix_constraint(c, p)
        linear = apply_substitution_to_map(storage, nl_map, subs, p)
        no_rounds -= 1
        apply_round = len(linear) > 0 and no_rounds > 0

    for c in linear:
        sigs = take_cloned_signals(c)
        cid = len(storage)
        storage.append(c)
        for s in sigs:
            nl_map.setdefault(s, []).append(cid)
    for c in lconst:
        fix_constraint(c, p)
        sigs = take_cloned_signals(c)
        cid = len(storage)
        storage.append(c)
        for s in sigs:
            nl_map.setdefault(s, []).append(cid)

    storage = [c for c in storage if not is_empty(c)]
    signal_map = rebuild_witness(sys_.max_signal, deleted, forbidden, nl_map, True)
    max_value_input = sys_.n_pub_out + sys_.n_pub_in + sys_.n_priv_in
    deleted_inputs = sum(1 for s in deleted if sys_.n_pub_out + 1 <= s <= max_value_input)
    return Result(storage, signal_map, sys_.n_priv_in - deleted_inputs, log or [])


# ----------------------------------------------------------------- formats
def field_size_bytes(p: int) -> int:
    """r1cs_porting.rs:6-10."""
    bits = p.bit_length()
    return bits // 8 if bits % 64 == 0 else (bits // 64 + 1) * 8


def _le_key(k: int) -> bytes:
    """BigInt::from(k).to_bytes_le().1 (zero -> [0])."""
    if k == 0:
        return b"\x00"
    return k.to_bytes((k.bit_length() + 7) // 8, "little")


def _lc_block(m: Map, fs: int) -> bytes:
    """r1cs_writer.rs:49-72: keys sorted by their LE byte strings."""
    out = [struct.pack("<I", len(m))]
    for kb in sorted(_le_key(k) for k in m):
        k = int.from_bytes(kb, "little")
        out.append(kb + b"\x00" * (4 - len(kb)))
        v = m[k]
        vb = b"\x00" if v == 0 else v.to_bytes((v.bit_length() + 7) // 8, "little")
        out.append(vb + b"\x00" * (fs - len(vb)))
    return b"".join(out)


def write_r1cs_bytes(p, constraints: List[Con], n_wires, n_pub_out, n_pub_in, n_priv_in,
                     n_labels, wire_to_label: List[int], gates=None) -> bytes:
    """constraint_list/src/r1cs_porting.rs:4-124 + r1cs_writer.rs: 3 sections, or 5 with custom
    gates -- `gates` = (section 4 bytes, [(gate index, [wires])]) written by
    write_custom_gates_usages / write_custom_gates_applications (r1cs_writer.rs:358-450)."""
    fs = field_size_bytes(p)
    body = b"".join(_lc_block(c.a, fs) + _lc_block(c.b, fs) + _lc_block(c.c, fs)
                    for c in constraints)
    sec_cons = struct.pack("<I", 2) + struct.pack("<Q", len(body)) + body
    hdr = (struct.pack("<I", fs) + p.to_bytes(fs, "little") +
           struct.pack("<IIIIQI", n_wires, n_pub_out, n_pub_in, n_priv_in, n_labels,
                       len(constraints)))
    sec_hdr = struct.pack("<I", 1) + struct.pack("<Q", len(hdr)) + hdr
    w2l = b"".join(struct.pack("<Q", x) for x in wire_to_label)
    sec_w2l = struct.pack("<I", 3) + struct.pack("<Q", len(w2l)) + w2l
    if gates is None:
        return b"r1cs" + bytes([1, 0, 0, 0, 3, 0, 0, 0]) + sec_cons + sec_hdr + sec_w2l
    used, apps = gates
    body5 = struct.pack("<I", len(apps)) + b"".join(
        struct.pack("<II", gi, len(sig)) + b"".join(struct.pack("<Q", x) for x in sig) for gi, sig in apps)
    sec4 = struct.pack("<IQ", 4, len(used)) + used
    sec5 = struct.pack("<IQ", 5, len(body5)) + body5
    return b"r1cs" + bytes([1, 0, 0, 0, 5, 0, 0, 0]) + sec_cons + sec_hdr + sec_w2l + sec4 + sec5


def apply_correspondence(c: Con, sm: Dict[int, int]) -> Con:
    """algebra.rs:1037-1048 + apply_raw_correspondence (:1245-1264)."""
    def f(m):
        return {(k if k == CONST else sm[k]): v for k, v in m.items()}
    return Con(f(c.a), f(c.b), f(c.c))


def result_to_r1cs(sys_: System, res: Result) -> bytes:
    wires = len(res.signal_map)
    w2l = [0] * wires
    for k, v in res.signal_map.items():
        w2l[v] = k
    cons = [apply_correspondence(c, res.signal_map) for c in res.constraints]
    gates = None
    if sys_.gates is not None:  # r1cs_porting.rs:90-107: signals through the SignalMap (unwrap)
        used, apps = sys_.gates
        gates = (used, [(gi, [res.signal_map[x] for x in sig]) for gi, sig in apps])
    return write_r1cs_bytes(sys_.p, cons, wires, sys_.n_pub_out, sys_.n_pub_in, sys_.n_priv_in,
                            sys_.max_signal, w2l, gates)


def result_to_sym(sym_lines: List[Tuple[int, int, int, str]], res: Result) -> str:
    """sym_porting.rs:5-37: the O0 sym lines with the witness column remapped (-1 = removed)."""
    out = []
    for orig, _w, node, name in sym_lines:
        w = res.signal_map.get(orig, -1)
        out.append(f"{orig},{w},{node},{name}\n")
    return "".join(out)


def read_r1cs_bytes(data: bytes) -> Tuple[System, dict]:
    """Minimal .r1cs reader (the --O0 export, CS-4); sections in any order."""
    assert data[:4] == b"r1cs"
    nsec = struct.unpack_from("<I", data, 8)[0]
    off = 12
    secs = {}
    for _ in range(nsec):
        t, sz = struct.unpack_from("<IQ", data, off)
        off += 12
        secs.setdefault(t, (off, sz))
        off += sz
    ho, _ = secs[1]
    fs = struct.unpack_from("<I", data, ho)[0]
    p = int.from_bytes(data[ho + 4: ho + 4 + fs], "little")
    n_wires, n_out, n_pub, n_prv, n_labels, n_cons = struct.unpack_from("<IIIIQI", data, ho + 4 + fs)
    co, _ = secs[2]
    rows = []
    o = co
    for _ in range(n_cons):
        lcs = []
        for _ in range(3):
            n = struct.unpack_from("<I", data, o)[0]
            o += 4
            m = {}
            for _ in range(n):
                k = struct.unpack_from("<I", data, o)[0]
                v = int.from_bytes(data[o + 4: o + 4 + fs], "little")
                o += 4 + fs
                m[k] = v
            lcs.append(m)
        rows.append(Con(*lcs))
    hdr = dict(fs=fs, n_wires=n_wires, n_labels=n_labels, n_cons=n_cons)
    forb = {0} | set(range(1, n_out + n_pub + 1))
    gates = None
    if 4 in secs or 5 in secs:
        used = data[secs[4][0]: secs[4][0] + secs[4][1]] if 4 in secs else struct.pack("<I", 0)
        apps = []
        if 5 in secs:
            o = secs[5][0]
            (na,) = struct.unpack_from("<I", data, o)
            o += 4
            for _ in range(na):
                gi, ns = struct.unpack_from("<II", data, o)
                o += 8
                sig = list(struct.unpack_from(f"<{ns}Q", data, o))
                o += 8 * ns
                apps.append((gi, sig))
                forb |= set(sig)  # map_to_constraint_list.rs:22-24: custom-gate signals are forbidden
        gates = (used, apps)
    return System(p, n_labels, n_out, n_pub, n_prv, forb, rows, gates), hdr


# ---------------------------------------------------------------- DAG -> constraint lists (8(f) rank 1)
@dataclass
class DagNode:
    """A DAG node as the flattening reads it (dag/src/lib.rs:141-176 Node): its constraints over
    node-local ids (0 = the constant), its own signals (is_local_signal), the custom-gate flag, and
    its edges in adjacency order as (goes_to, in_number) (dag/src/lib.rs:87-100 Edge)."""
    constraints: List[Con]
    locals: List[int]
    custom_gate: bool = False
    edges: List[Tuple[int, int]] = dc_field(default_factory=list)


def _offset_map(m: Map, off: int) -> Map:
    """apply_raw_offset (algebra.rs:1266-1277): every key but the constant moves by the offset."""
    return {(k if k == CONST else k + off): v for k, v in m.items()}


def flatten_dag(p: int, nodes: List[DagNode], main: int, n_pub_out: int, n_pub_in: int, n_priv_in: int,
                forbidden_main) -> Tuple[System, dict]:
    """dag/src/map_to_constraint_list.rs:111-150 (map) over the tree walk of map_tree (:12-44) with
    Tree::new / Tree::go_to_subtree (dag/src/lib.rs:35-85: main at offset 0 keeps every constraint, a
    subtree drops the empty ones and applies its offset), plus the non-linear rows in the
    EncodingIterator's DFS (constraint_list/src/lib.rs:65-108, state_utils.rs:14-35 over
    map_node_to_encoding's non_linear, map_to_constraint_list.rs:71-104).  Returns the System the
    Simplifier is built from (rows in DFS order) and the blocks as map() fills them."""
    ce, eq, lin, nl = [], [], [], []
    witness = [0]
    forbidden = set(forbidden_main)
    rows = []
    stack = [(main, 0, True)]
    while stack:  # pre-order, children in adjacency order
        nid, off, root = stack.pop()
        node = nodes[nid]
        for s in sorted(node.locals):
            witness.append(s + off)
            if node.custom_gate:
                forbidden.add(s + off)
        for c in node.constraints:
            if not root and is_empty(c):
                continue
            c = Con(_offset_map(c.a, off), _offset_map(c.b, off), _offset_map(c.c, off))
            rows.append(c)
            if is_constant_equality(c):
                ce.append(c)
            elif is_equality(c, p):
                eq.append(c)
            elif is_linear(c):
                lin.append(c)
            else:
                nl.append(c)
        for child, inn in reversed(node.edges):
            stack.append((child, off + inn, False))
    sys_ = System(p, len(witness), n_pub_out, n_pub_in, n_priv_in, forbidden, rows)
    return sys_, dict(cons_eq=ce, eq=eq, linear=lin, non_linear=nl, witness=witness)


def to_json_constraints(constraints: List[Con], sm: Dict[int, int]) -> list:
    """json_porting.rs:8-48 (numeric key order, decimal strings)."""
    out = []
    for c in constraints:
        c = apply_correspondence(c, sm)
        out.append([{str(k): str(m[k]) for k in sorted(m)} for m in (c.a, c.b, c.c)])
    return out

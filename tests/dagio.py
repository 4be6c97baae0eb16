"""Seeded random component DAGs for the flattening tests, with consistent
signal numbering: a template's own signals are 1..L, its k-th child's signals sit at
in_number + (1..size(child)) with in_number = L + the earlier children's sizes -- the numbering
circom's DAG uses (dag/src/lib.rs:179-220 add_input/add_output/add_intermediate, add_edge)."""
import random

import rsio

R = rsio.R


def gen_dag(seed: int, p: int, n_templates: int = 6, max_children: int = 3, empties: bool = False,
            custom_gates: bool = False, cons_per_template=(4, 14)):
    """-> (nodes, main, n_pub_out, n_pub_in, n_priv_in, forbidden_main)."""
    rng = random.Random(seed)
    nodes, size = [], []

    def coef():
        r = rng.random()
        return 1 if r < 0.3 else (p - 1 if r < 0.5 else rng.randrange(1, p))

    for t in range(n_templates):
        L = rng.randint(2, 7) if t < n_templates - 1 else rng.randint(3, 7)  # main: out, pub in, priv in
        kids = [rng.randrange(t) for _ in range(rng.randint(0 if t else 0, max_children if t else 0))]
        edges, off = [], L
        for ch in kids:
            edges.append((ch, off))
            off += size[ch]
        S = off
        size.append(S)
        sig = lambda: rng.randint(1, S)
        cons = []
        for _ in range(rng.randint(*cons_per_template)):
            r = rng.random()
            if r < 0.15:    # constant equality
                m = {sig(): coef()}
                if rng.random() < 0.7:
                    m[0] = coef()
                cons.append(R.Con({}, {}, m))
            elif r < 0.35:  # equality x = y
                x, y = sig(), sig()
                if x == y:
                    continue
                c = coef()
                cons.append(R.Con({}, {}, {x: c, y: (p - c) % p}))
            elif r < 0.65:  # linear
                m = {}
                for _ in range(rng.randint(3, 5)):
                    m[sig()] = coef()
                if rng.random() < 0.3:
                    m[0] = coef()
                cons.append(R.Con({}, {}, m))
            else:           # quadratic
                a = {sig(): coef()}
                b = {sig(): coef()}
                if rng.random() < 0.3:
                    b[sig()] = coef()
                c = {sig(): coef()}
                if rng.random() < 0.3:
                    c[0] = coef()
                cons.append(R.Con(a, b, c))
            if empties and rng.random() < 0.08:
                cons.append(R.Con({}, {}, {}))
        gate = custom_gates and t < n_templates - 1 and rng.random() < 0.3
        nodes.append(R.DagNode(cons, list(range(1, L + 1)), gate, edges))
    main = n_templates - 1
    n_out, n_pub, n_prv = 1, 1, 1
    forbidden = set(range(0, 1 + n_out + n_pub))
    return nodes, main, n_out, n_pub, n_prv, forbidden

#!/usr/bin/env python3
"""Debug probe: node2vec MH WEIGHT generation on a small RMAT graph vs the
oracle, and two device runs against each other (determinism)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import dynamicgraphrepresentationlearning_amd as W
    from oracle import oracle as O
    base = O.generate_batch_of_edges(40000, 1 << 12, 5, False, False)
    off, adj = O.csr_from_edges(1 << 11, base)
    kw = dict(walks_per_vertex=4, walk_length=40, model=1, paramP=0.5, paramQ=2.0, sampler_init=2,
              deterministic=False, seed=1234 + 2)
    runs = []
    for _ in range(2):
        g = W.WharfMH.from_csr(off, adj, config=W.WharfConfig(**kw))
        g.generate_initial_random_walks()
        runs.append(g.walks().copy())
        g.destroy()
    ref = O.Engine(off, adj, wpv=4, L=40, model=1, p=0.5, q=2.0, init=2, deterministic=False, seed=1234 + 2)
    ref.generate()
    rw = ref.walks()
    print("device runs identical:", np.array_equal(runs[0], runs[1]), int((runs[0] != runs[1]).sum()))
    bad = np.nonzero((runs[0] != rw).any(axis=1))[0]
    print("walks differing from oracle:", len(bad), "of", len(rw))
    for w in bad[:5]:
        p = int(np.nonzero(runs[0][w] != rw[w])[0][0])
        print(f"wid {w}: first diff at pos {p}: dev {runs[0][w][max(0,p-2):p+2]} ref {rw[w][max(0,p-2):p+2]}")
        cur, prev = int(rw[w][p - 1]), int(rw[w][p - 2]) if p >= 2 else -1
        d = int(off[cur + 1] - off[cur])
        print(f"   cur {cur} deg {d}, prev {prev} deg {int(off[prev+1]-off[prev]) if prev >= 0 else -1}")


if __name__ == "__main__":
    main()

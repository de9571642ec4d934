"""Card-set ownership statistics on a real beam (analysis for the N>1 protocol; uses the C oracle).

Runs the oracle's seeded solve to a saturated turn, then for world 8: parents per card-set owner (load
balance), raw children that keep the parent's card set (takes: claimed where generated) vs buys, and buys
whose new card set the parent's rank owns anyway.
Usage: python profiles/analysis/cardset_stats.py HEUR WIDTH TURN
"""
import random
import sys
import time

import numpy as np

sys.path[:0] = ['oracle', 'splendor-rl-gym_amd']
import oracle_c  # noqa: E402

M64 = (1 << 64) - 1
CARDS_HI = (1 << 26) - 1


def mix64(x):
    x = x.copy()
    x ^= x >> np.uint64(33)
    x *= np.uint64(0xff51afd7ed558ccd)
    x ^= x >> np.uint64(33)
    x *= np.uint64(0xc4ceb9fe1a85ec53)
    x ^= x >> np.uint64(33)
    return x


def cs_owner(lo, hi, world):
    h = mix64(lo ^ mix64((hi & np.uint64(CARDS_HI)) + np.uint64(0x9E3779B97F4A7C15)))
    return ((h >> np.uint64(40)) % np.uint64(world)).astype(np.int64)


def main():
    heur, W, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    world = 8
    random.seed(0)
    o = oracle_c.OracleSolve(15, use_heuristic=True, heuristic_name=heur, beam_width=W,
                             mt_state625=random.getstate()[1])
    t0 = time.time()
    for _ in range(T):
        s = o.step()
    lo, hi, par, key = o.turn_arrays(T)
    print(f'turn {T}: {len(lo)} parents ({time.time() - t0:.0f} s)', flush=True)
    n = len(lo)
    own = cs_owner(lo, hi, world)
    csets = lo.astype(object) * 0
    cs = np.unique(np.stack([lo, hi & np.uint64(CARDS_HI)], 1), axis=0)
    per = np.bincount(own, minlength=world)
    print(f'distinct card sets {len(cs)}; parents per owner: {per.tolist()}; max/mean {per.max() / per.mean():.3f}')
    L = oracle_c.lib()
    olo = np.zeros(256, np.uint64)
    ohi = np.zeros(256, np.uint64)
    okey = np.zeros(256, np.uint64)
    step = max(1, n // 400000)
    raw = take = buy_local = buy_remote = 0
    raw_per = np.zeros(world, np.int64)
    recv_per = np.zeros(world, np.int64)
    for i in range(0, n, step):
        k = L.oc_successors(int(lo[i]), int(hi[i]), olo, ohi, okey)
        c = olo[:k]
        ch = ohi[:k] & np.uint64(CARDS_HI)
        same = (c == lo[i]) & (ch == (hi[i] & np.uint64(CARDS_HI)))
        raw += k
        raw_per[own[i]] += k
        take += int(same.sum())
        if (~same).any():
            bo = cs_owner(c[~same], ohi[:k][~same], world)
            bl = int((bo == own[i]).sum())
            buy_local += bl
            buy_remote += int((~same).sum()) - bl
            np.add.at(recv_per, bo[bo != own[i]], 1)
    print(f'sampled every {step}: raw {raw}, same card set (takes) {take / raw:.3f}, buys {1 - take / raw:.3f} '
          f'(local {buy_local / raw:.3f}, remote {buy_remote / raw:.3f} of raw)')
    print(f'raw per owner max/mean {raw_per.max() / raw_per.mean():.3f}; records received per owner max/mean '
          f'{recv_per.max() / max(recv_per.mean(), 1):.3f}')
    o.close()


if __name__ == '__main__':
    main()

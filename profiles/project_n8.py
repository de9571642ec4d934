#!/usr/bin/env python3
"""N=8 projection of the sharded step from one-GPU measurements.

Inputs: a per-rank phase table (profiles/sharded_table.py --out: serialised world-8 traces on one GPU, each
rank's kernels alone on the device = its own GPU's device time) and a bench line of the same run
(bench_dist.py: exchange_MB_per_step_rank0 = bytes rank 0 sent to other ranks per step, by exchange).

Model per rank and step: device time (the table's engine-stream total; the noise side stream overlaps) plus
the exchanges that sit on the critical path at an effective all_to_all rate B per GPU (xGMI: 7 links per
MI355X; RCCL's all_to_all rate is unmeasured here — one GPU per box — so B is a parameter), plus a fixed
latency per collective round.  The records travel in P parts beside the key pass: part j leaves when its key pass
is done, so what the claims wait for beyond the key pass is max(x / P, x - kp (P - 1) / P) for a transfer time x
and key pass kp (round 5: the last part's transfer always counts — earlier rounds counted only max(0, x - kp)).
Every other exchange counts in full.
Round 6: the latency is two terms.  Host metadata rounds (the turn sync and each part's counts: 1 +
parts per step, host all_gathers) at --host-lat-us, measured on CPU by profiles/gloo_latency.py (shared memory, the
default since round 6: 8 us a round at world 8; gloo's TCP ring: 1.3-6 ms on an 8-core host) — the JSON it wrote can be
given as --host-lat-json.  Device collective rounds (RCCL: the select's 8 all_reduces, the tie and count gathers, the
parts' and the answers' all_to_alls, the kept records' counts and segments: ~20 per step, counted from SB_DIST_HOSTPROF
in profiles/r6/) at --lat-us, which stays an assumption: one GPU per box here.
    python3 profiles/project_n8.py TABLE.json BENCH.json [--B 250,400,600] [--lat-us 30] [--rounds 20]
                                   [--host-lat-json profiles/r6/gloo_latency_w8_container.json | --host-lat-us 8]
"""
import argparse
import json

OVERLAPPED = {'records'}   # exchanged part by part while the key pass runs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('table')
    ap.add_argument('bench')
    ap.add_argument('--B', default='250,400,600', help='effective all_to_all GB/s per GPU')
    ap.add_argument('--lat-us', type=float, default=30.0, help='latency per collective round (us)')
    ap.add_argument('--rounds', type=float, default=None, help='device collective rounds per step on the critical path '
                    '(default: the bench line\'s counted collectives_per_step_rank0, else 20)')
    ap.add_argument('--host-lat-us', type=float, default=None, help='host metadata all_gather latency (us)')
    ap.add_argument('--host-lat-json', default=None, help='profiles/gloo_latency.py output: its shared-memory chain')
    ap.add_argument('--host-gloo', action='store_true', help='with --host-lat-json: the gloo chain instead')
    ap.add_argument('--single-ms', type=float, default=4.548, help='one GPU ms/step (BENCH_r04: 4.548)')
    ap.add_argument('--balanced-kept', action='store_true',
                    help='kept records as if every rank sent 7/8 of W x 32 B (a protocol whose kept records are produced '
                         'evenly); by default rank 0, which sends the most, as measured')
    ap.add_argument('--W', type=float, default=4e6, help='parents per rank')
    ap.add_argument('--parts', type=int, default=4, help='exchange parts of the key pass (SB_DIST_PARTS)')
    ap.add_argument('--device-ms', type=float, default=None,
                    help='device time per rank and step from another measurement (e.g. the world-1 key-pass run, '
                         'profiles/busy_union.py) instead of the table\'s serialised total')
    a = ap.parse_args()
    host_lat = a.host_lat_us
    if a.host_lat_json:
        hj = json.load(open(a.host_lat_json))
        host_lat = hj['part_counts_chain_us_max_rank' if a.host_gloo else 'shm_part_counts_chain_us_max_rank']
    host_rounds = 1 + a.parts
    t = json.load(open(a.table))
    b = [json.loads(l) for l in open(a.bench) if l.startswith('{')][-1]
    counted = b.get('collectives_per_step_rank0')
    rounds_src = 'assumed'
    if a.rounds is None and counted:   # counted by Comm in the traced run
        a.rounds, host_rounds, rounds_src = counted['device'], counted['host'], 'counted'
    elif a.rounds is None:
        a.rounds = 20
    mean = t.get('robust_mean_ms', t['mean_ms'])   # launches that waited on another rank's work capped
    dev = mean['device total (engine stream)'] if a.device_ms is None else a.device_ms
    keypass = mean.get('expand', 0.0)
    x = dict(b.get('exchange_MB_per_step_rank0', {}))
    if a.balanced_kept and 'kept records' in x:
        x['kept records'] = a.W * 32 * 7 / 8 / 1e6
    print(f'device per rank (serialised world-{t["world"]} traces, mean of ranks): {dev:.3f} ms; key pass {keypass:.3f} ms')
    print('exchange per rank and step (MB sent to other ranks):', {k: round(v, 1) for k, v in x.items()})
    out = {'device_ms': dev, 'exchange_MB': x, 'projection': [],
           'latency_model': {'device_rounds': a.rounds, 'rounds_source': rounds_src, 'device_lat_us': a.lat_us,
                             'host_rounds': host_rounds,
                             'host_lat_us': host_lat}}
    if host_lat is not None:
        print(f'latency: {a.rounds} device collective rounds ({rounds_src}) x {a.lat_us} us (assumed) + {host_rounds} host '
              f'metadata rounds x {host_lat} us (measured)')
    for B in [float(v) for v in a.B.split(',')]:
        crit = sum(v for k, v in x.items() if k not in OVERLAPPED) / B          # MB / (GB/s) = ms
        over = sum(v for k, v in x.items() if k in OVERLAPPED) / B
        P = a.parts
        exposed_rec = max(over / P, over - keypass * (P - 1) / P) if over > 0 else 0.0
        lat = a.rounds * a.lat_us / 1e3 + (host_rounds * host_lat / 1e3 if host_lat is not None else 0.0)
        step = dev + crit + exposed_rec + lat
        gps = 8 * a.W / (step * 1e-3) / 1e9
        row = {'B_GBps': B, 'critical_exchange_ms': round(crit, 3), 'records_exposed_ms': round(exposed_rec, 3),
               'latency_ms': round(lat, 3), 'step_ms': round(step, 3), 'G_states_per_s_N8': round(gps, 2),
               'speedup_vs_1gpu': round(a.single_ms / step * 8, 2)}
        out['projection'].append(row)
        print(f'B={B:5.0f} GB/s: step {step:.3f} ms = device {dev:.3f} + exchanges {crit:.3f} (+{exposed_rec:.3f} '
              f'records beyond the key pass) + latency {lat:.3f} -> {gps:.2f} G states/s at N=8, '
              f'{row["speedup_vs_1gpu"]:.2f}x one GPU ({a.single_ms} ms)')
    print(json.dumps(out))


if __name__ == '__main__':
    main()

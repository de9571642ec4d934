"""Beam sharding across GPUs: one process per GPU, torch.distributed (RCCL over xGMI) for the exchanges.

The global queue of a turn is split into contiguous rank ranges (rank r holds global queue
positions [off_r, off_r + n_r)), so the (parent rank, ordinal) order that decides first occurrence
(src/solver.py:446-450) and the noise order (sorted() calls its key in next_queue order,
src/solver.py:452-456) stay global.  One step, per rank:

  turn sync one all_gather per turn of (slice size, first local position per pts): slice offsets and
            the goal check (src/solver.py:438-445)
  expand    every successor of the local parents has an owner (mix64(key) top bits mod world); the
            ones this rank owns are claimed in its shard of the global visited set during the
            expansion, every other one becomes a record (key), grouped by owner in (parent, ordinal)
            order; one all_gather of the per-owner counts sizes the exchange
  dedup     all_to_all of the keys to their owners; records arrive source rank by source rank, so
            (source rank, record index) is the global (parent rank, ordinal) order: the owner claims
            with tag = turn | source | index (its own children: turn | rank | parent | move) and
            answers one bit per record (first occurrence or not); all_to_all back
  offsets   all_gather of per-rank unique counts -> this rank's next_queue offset k_off
  emit      survivors' states + scores; noise = accepted MT draw (consumed + k_off + k), from the
            sharded MT19937 stream (ShardNoise)
  select    top-W of all scores, stable (score desc, next_queue order asc), on the device: MSB radix
            select with all_reduce(SUM) of 1024-bin histograms per distinct prefix per pass, for the
            keep boundary and the world-1 split boundaries of the kept set; ties at the keep
            boundary are taken in global order via all_gather of per-rank tie counts
  rebalance all_to_all of the kept 32-byte records to their destination range; the receiver
            stable-sorts by score (records arrive in source order = global next_queue order)

The backend supplies the per-rank compute (HipBackend: libsplendor_beam.so; tests: a Python
reference backend).  All results are bit-identical to the single-GPU engine and the oracle.
"""
from __future__ import annotations

import contextlib
import os
import time

import numpy as np
import torch
import torch.distributed as dist

_PHASES = os.environ.get('SB_DIST_PHASES') == '1'   # diagnostic: host wall time per protocol phase

NONE32 = 0xFFFFFFFF
BIG = (1 << 62)


# grouped kept records on the rebalance's wire (key ownership, world > 1): SB_DIST_GKR=0 sends the 20-byte records
GKR = os.environ.get('SB_DIST_GKR', '1') != '0'
# block-cyclic slices (key ownership with global-order claims, beam search): the next beam is dealt to the ranks in
# world x parts blocks, block b to rank b % world as its part b // world.  Part j of every rank is then one contiguous
# range of the global order, after every earlier part, so its claims run as soon as it has arrived (beside the next
# parts' key pass), and every rank holds parents of every score level (the kept records leave every rank about evenly).
# SB_DIST_BC=0: contiguous rank ranges (claims after the last part)
BC = os.environ.get('SB_DIST_BC', '1') != '0'

class ShmMeta:
    """Host all_gather of small int64 vectors among the ranks of one node through shared memory (the step's metadata:
    the turn sync, each exchange part's per-owner counts).  gloo's TCP ring took 170 us at world 2 and 6 ms at world 8
    on an 8-core host (profiles/gloo_latency.py); here a rank writes its vector into its slot, then its round number,
    and reads every slot once every rank's number has reached the round: a few microseconds plus the ranks' skew.

    Slots alternate by round parity: a rank writing round k + 1 knows every rank finished reading round k - 1 (each
    published round k only after that).  Ordering: x86-64 keeps stores in order and loads in order (TSO), so the data
    a rank stores before its round number is visible to any rank that sees the number."""

    SLOT = 1024   # int64 per rank and slot (the turn sync is 257 + parts)
    TIMEOUT_S = 600.0

    def __init__(self, rank, world, group):
        from multiprocessing import shared_memory
        import platform
        if platform.machine() not in ('x86_64', 'AMD64'):
            raise RuntimeError('ShmMeta relies on x86-64 store/load ordering')
        self.rank, self.world = rank, world
        nbytes = 8 * (world * 8 + 2 * world * self.SLOT)
        name = [None]
        if rank == 0:
            self._shm = shared_memory.SharedMemory(create=True, size=nbytes)
            self._shm.buf[:nbytes] = bytes(nbytes)
            name[0] = self._shm.name
        dist.broadcast_object_list(name, src=0, group=group)
        if rank != 0:   # attach without registering: the creator owns (and unlinks) the segment
            from multiprocessing import resource_tracker
            reg = resource_tracker.register
            resource_tracker.register = lambda *a, **k: None
            try:
                self._shm = shared_memory.SharedMemory(name=name[0])
            finally:
                resource_tracker.register = reg
        a = np.ndarray((world * 8 + 2 * world * self.SLOT,), dtype=np.int64, buffer=self._shm.buf)
        self.seq = a[:world * 8].reshape(world, 8)   # [r, 0]: the last round rank r published (a line per rank)
        self.data = a[world * 8:].reshape(2, world, self.SLOT)
        self.round = 0
        dist.barrier(group=group)   # every rank attached before the creator may unlink
        if rank == 0:
            self._shm.unlink()       # the mapping lives on in every process; nothing left under /dev/shm

    def allgather(self, arr: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(arr, dtype=np.int64)
        if len(a) > self.SLOT:
            raise ValueError(f'ShmMeta: {len(a)} values exceed the slot ({self.SLOT})')
        self.round += 1
        k = self.round
        slot = self.data[k & 1]
        slot[self.rank, :len(a)] = a
        self.seq[self.rank, 0] = k
        spins, t0 = 0, None
        while int(self.seq[:, 0].min()) < k:
            spins += 1
            if spins > 64:
                os.sched_yield()
                if spins % 4096 == 0:   # a rank that died would leave the others spinning
                    t0 = t0 or time.monotonic()
                    if time.monotonic() - t0 > self.TIMEOUT_S:
                        raise RuntimeError(f'ShmMeta: round {k} incomplete after {self.TIMEOUT_S} s '
                                           f'(rounds seen: {self.seq[:, 0].tolist()})')
        return slot[:, :len(a)].copy()

    def close(self):
        try:
            self.seq = self.data = None
            self._shm.close()
        except Exception:
            pass


# block-cyclic slices: part 0's blocks of the next beam, relative to the other parts' (SB_DIST_P0)
P0 = float(os.environ.get('SB_DIST_P0', '1.0'))

# host metadata over shared memory when every rank is on this node (SB_DIST_SHM=0: the gloo group)
SHM = os.environ.get('SB_DIST_SHM', '1') != '0'


class Comm:
    """torch.distributed helpers; gloo works on CPU tensors (device tensors are staged)."""

    def __init__(self, device: torch.device):
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.device = device
        self.backend = dist.get_backend()
        self.cpu_coll = self.backend == 'gloo'
        # host-side metadata (the turn sync: slice sizes + goal tables) goes over a gloo group: it runs
        # while the expansion occupies every CU, which a device collective would have to wait for
        self.meta = dist.new_group(backend='gloo') if self.world > 1 else None
        # ... and, when every rank runs on this node (one process per GPU of one MI355X node), over shared memory
        self.shm = None
        local = int(os.environ.get('LOCAL_WORLD_SIZE', self.world))
        if self.world > 1 and SHM and local == self.world:
            try:
                self.shm = ShmMeta(self.rank, self.world, self.meta)
            except (RuntimeError, OSError):
                self.shm = None
        self.devlock = None   # profiling (SerializedBackend.lock): gloo's staging copies under the device lock
        self.xbytes = {}      # bytes this rank sent to other ranks, per exchange (DistSolve.step hands them out)
        self.ncoll = 0        # device-group collectives issued (the step's latency rounds; DistSolve.step resets them)
        self.nhost = 0        # host metadata all_gathers (shared memory or the gloo group)

    def acct(self, what, nbytes):
        self.xbytes[what] = self.xbytes.get(what, 0) + int(nbytes)

    def _remote(self, pieces):
        return sum(int(p.numel()) * p.element_size() for o, p in enumerate(pieces) if o != self.rank)

    def _cp(self, fn):
        """A device copy of the gloo staging; under the profiling device lock when one is set."""
        if self.devlock is None:
            return fn()
        with self.devlock():
            out = fn()
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            return out

    def _to(self, t):
        return self._cp(lambda: t.cpu()) if self.cpu_coll else t

    def _back(self, t):
        return self._cp(lambda: t.to(self.device)) if self.cpu_coll and self.device.type != 'cpu' else t

    def allreduce(self, arr: np.ndarray, op) -> np.ndarray:
        t = self._to(self._cp(lambda: torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64)).to(self.device)))
        self.ncoll += 1
        dist.all_reduce(t, op=op)
        return t.cpu().numpy()

    def _gather_flat(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's equal-shape tensor, concatenated rank-major in one flat tensor: one collective
        (all_gather_into_tensor), so the host reads it back with one copy instead of one per rank."""
        s = self._to(t).reshape(-1)
        if self.world == 1:
            return s
        out = torch.empty(self.world * s.numel(), dtype=s.dtype, device=s.device)
        self.ncoll += 1
        dist.all_gather_into_tensor(out, s)
        return out

    def allgather_int(self, v: int) -> np.ndarray:
        if self.world == 1:
            return np.array([int(v)], dtype=np.int64)
        t = self._cp(lambda: torch.tensor([int(v)], dtype=torch.int64, device=self.device))
        return self._gather_flat(t).cpu().numpy().astype(np.int64)

    def gather_dev(self, t: torch.Tensor) -> np.ndarray:
        """Every rank's equal-shape device tensor, concatenated rank-major, on the host (one wait)."""
        return self._gather_flat(t).cpu().numpy()

    def alltoall_counts_dev(self, counts: torch.Tensor) -> tuple[np.ndarray, np.ndarray]:
        """(send counts, receive counts) on the host from a device tensor of send counts: one wait."""
        if self.world == 1:
            c = counts.cpu().numpy()
            return c, c
        send = self._to(counts.reshape(-1))   # world x k counts: k per destination (equal splits)
        recv = torch.empty_like(send)
        self.ncoll += 1
        dist.all_to_all_single(recv, send)
        both = torch.cat([send, recv]).cpu().numpy()
        return both[:send.numel()], both[send.numel():]

    def alltoall_counts(self, counts: np.ndarray) -> np.ndarray:
        send = self._to(torch.from_numpy(np.ascontiguousarray(counts, dtype=np.int64)).to(self.device))
        recv = torch.empty_like(send)
        self.ncoll += 1
        dist.all_to_all_single(recv, send)
        return recv.cpu().numpy()

    def alltoall(self, send: torch.Tensor, send_counts, recv_counts, what='other') -> torch.Tensor:
        row = send.element_size() * (int(send[0].numel()) if send.dim() > 1 and send.shape[0] else 1)
        self.acct(what, row * (int(sum(send_counts)) - int(send_counts[self.rank])))
        s = self._to(send)
        r = torch.empty((int(sum(recv_counts)),) + tuple(send.shape[1:]), dtype=send.dtype, device=s.device)
        self.ncoll += 1
        dist.all_to_all_single(r, s, [int(x) for x in recv_counts], [int(x) for x in send_counts])
        return self._back(r)

    def alltoall_pieces(self, pieces, recv_sizes, what='other', out=None):
        """Start an all_to_all of pieces[o] (views, any layout) to rank o; returns (receive buffer,
        handle).  RCCL runs it asynchronously on its own stream; wait(handle) orders this rank's stream
        after it.  gloo (no list all_to_all) packs the pieces and completes at once.  out: a 1-D view to
        receive into (sum(recv_sizes) elements), else a new buffer."""
        self.acct(what, self._remote(pieces))
        if out is None:
            out = torch.empty(int(sum(recv_sizes)), dtype=pieces[0].dtype, device=pieces[0].device)
        if self.cpu_coll:
            send = self._cp(lambda: torch.cat([p.cpu() for p in pieces]))
            r = torch.empty(int(sum(recv_sizes)), dtype=send.dtype)
            self.ncoll += 1
            dist.all_to_all_single(r, send, [int(x) for x in recv_sizes], [int(p.numel()) for p in pieces])
            self._cp(lambda: out.copy_(r.to(out.device)))
            return out, None
        outs = list(out.split([int(x) for x in recv_sizes]))
        self.ncoll += 1
        return out, dist.all_to_all(outs, list(pieces), async_op=True)

    def alltoall_into(self, pieces, outs, what='other'):
        """all_to_all of pieces[o] (views) to rank o, received straight into the views outs[o]."""
        self.acct(what, self._remote(pieces))
        if self.cpu_coll:
            send = self._cp(lambda: torch.cat([p.cpu() for p in pieces]))
            rows = [int(o.shape[0]) for o in outs]
            r = torch.empty((sum(rows),) + tuple(outs[0].shape[1:]), dtype=send.dtype)
            self.ncoll += 1
            dist.all_to_all_single(r, send, rows, [int(p.shape[0]) for p in pieces])

            def back():
                for o, x in zip(outs, r.split(rows)):
                    o.copy_(x.to(o.device))
            self._cp(back)
            return
        self.ncoll += 1
        dist.all_to_all(list(outs), list(pieces))

    @staticmethod
    def wait(handle):
        if handle is not None:
            handle.wait()

    def allreduce_tensor(self, t: torch.Tensor, op=dist.ReduceOp.SUM, what='select all_reduce'):
        """In-place reduction over ranks of a tensor on this rank's device (no host wait with RCCL)."""
        if self.world == 1:
            return
        self.acct(what, 2 * (self.world - 1) * t.numel() * t.element_size() // self.world)   # ring volume
        if self.cpu_coll:
            x = self._cp(lambda: t.cpu())
            self.ncoll += 1
            dist.all_reduce(x, op=op)
            self._cp(lambda: t.copy_(x.to(t.device)))
        else:
            self.ncoll += 1
            dist.all_reduce(t, op=op)

    def allgather_array(self, arr: np.ndarray, host: bool = False) -> np.ndarray:
        """(world, len) int64 array of every rank's equal-length int vector (host: over the gloo metadata
        group, no device work)."""
        a = np.ascontiguousarray(arr, dtype=np.int64)
        if self.world == 1:   # nothing to exchange: no device round trip
            return a.reshape(1, len(a))
        if host:
            if self.shm is not None and len(a) <= ShmMeta.SLOT:
                self.nhost += 1
                return self.shm.allgather(a)
            t = torch.from_numpy(a)
            out = [torch.empty_like(t) for _ in range(self.world)]
            self.nhost += 1
            dist.all_gather(out, t, group=self.meta)
            return torch.stack(out).numpy()
        t = self._cp(lambda: torch.from_numpy(a).to(self.device))
        return self._gather_flat(t).cpu().numpy().reshape(self.world, len(a))

    def allgather_var(self, arr: np.ndarray) -> np.ndarray:
        """Every rank's int64 vector of any length, concatenated rank-major (host, gloo metadata group)."""
        a = np.ascontiguousarray(arr, dtype=np.int64)
        if self.world == 1:
            return a
        n = self.allgather_array(np.array([len(a)]), host=True)[:, 0]
        pad = np.zeros(int(n.max()) if len(n) else 0, np.int64)
        pad[:len(a)] = a
        out = self.allgather_array(pad, host=True) if len(pad) else np.zeros((self.world, 0), np.int64)
        return np.concatenate([out[r, :int(n[r])] for r in range(self.world)])

    def allgather_tensor(self, t: torch.Tensor) -> torch.Tensor:
        """(world, *t.shape): every rank's equal-shape tensor, on this rank's device."""
        return self._back(self._gather_flat(t).reshape((self.world,) + tuple(t.shape)))

    def broadcast_ints(self, vals, src: int) -> list[int]:
        t = self._to(self._cp(lambda: torch.tensor([int(v) for v in vals], dtype=torch.int64, device=self.device)))
        self.ncoll += 1
        dist.broadcast(t, src)
        return [int(x) for x in t.cpu().tolist()]

    def barrier(self):
        self.ncoll += 1
        dist.barrier()


def _u64_to_i64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


class ShardNoise:
    """The randint(1,100) stream without replicated generation.

    The k-th next_queue entry scores with the k-th accepted MT19937 draw (src/solver.py:452-456);
    rank r emits entries [k_off, k_off + n_loc) of each turn.  The raw stream after the lead block is
    cut into chunks of P producer segments; rank r generates chunks c = r (mod world) in count-only
    mode, keeping a checkpoint window every ck twists (a sub-segment) on its device, and every rank
    all-gathers the per-sub-segment accepted counts.  Once the turn's offsets are known every rank
    knows every rank's draw range, so the generating ranks send the windows of the sub-segments each
    rank needs in one all_to_all (sizes computed identically everywhere, no request round), and each
    rank regenerates just those sub-segments.  Per step a rank generates about 2/world of the stream.
    """

    def __init__(self, backend, comm: Comm):
        self.b, self.c = backend, comm
        info = backend.noise_info()
        self.P, self.S, self.nslots = int(info[0]), int(info[5]), int(info[6])
        self.gen_total = int(info[2])   # accepted draws available (global index), the lead block first
        self.round = 0                  # chunk rounds launched (one chunk per rank each)
        self.chunks = []                # (first global accepted index, cumulative counts (P*S+1), rank, slot)
        self.pending = None             # (slot, counts) of a round launched but not yet gathered

    def _launch(self):
        slot = self.round % self.nslots
        if any(ch[3] == slot for ch in self.chunks):
            raise RuntimeError('noise checkpoint slot still holds unconsumed draws')
        self.pending = (slot, self.b.noise_chunk(slot))
        self.round += 1

    def _collect(self):
        """All-gather the sub-segment counts of the round launched by _launch (every rank one chunk)."""
        c, b = self.c, self.b
        slot, counts = self.pending
        self.pending = None
        b.noise_sync()
        allc = c.allgather_tensor(counts).cpu().numpy().astype(np.int64)   # (world, P*S)
        for r in range(c.world):   # chunk order: this round's chunk of rank 0, 1, ...
            cum = np.concatenate([[0], np.cumsum(allc[r])]).astype(np.int64)
            self.chunks.append((self.gen_total, cum, r, slot))
            self.gen_total += int(cum[-1])

    @staticmethod
    def _subsegs_multi(s0, cum, rr):
        """Non-empty sub-segments of a chunk (first global accepted index s0, cumulative counts cum) holding draws of
        any of the ranges rr ((k, 2): [a, e) global indices), sorted: one pair of searchsorted calls for all of them
        (the step's host path waits on this between the apply and the emission)."""
        a, e = rr[:, 0] - s0, rr[:, 1] - s0
        keep = (e > a) & (e > 0) & (a < cum[-1])
        if not keep.any():
            return np.zeros(0, np.int64)
        a, e = a[keep], e[keep]
        j0 = np.maximum(np.searchsorted(cum, a, side='right') - 1, 0)
        j1 = np.minimum(np.searchsorted(cum, e, side='left'), len(cum) - 1)
        if len(a) == 1:
            js = np.arange(j0[0], j1[0], dtype=np.int64)
        else:   # the ranges' sub-segment intervals merged (a rank's blocks are few: a Python pass), then enumerated
            segs = []
            for x, y in sorted(zip(j0.tolist(), j1.tolist())):
                if segs and x <= segs[-1][1]:
                    segs[-1][1] = max(segs[-1][1], y)
                elif y > x:
                    segs.append([x, y])
            js = (np.concatenate([np.arange(x, y, dtype=np.int64) for x, y in segs]) if segs
                  else np.zeros(0, np.int64))
        return js[cum[js + 1] > cum[js]]

    def prepare(self, A: int, N: int, all_n: np.ndarray, blocks: np.ndarray | None = None):
        """Make this rank's accepted draws [A + k_off, A + k_off + n_loc) available to its emission (k_off = the
        next_queue entries of the ranks before it).  blocks (block-cyclic slices, (world, parts) entries per block):
        this rank's draws are those of its blocks' global next_queue ranges, placed at local positions k_off + its
        earlier blocks' entries."""
        c, b = self.c, self.b
        # the round in flight is gathered only once its draws are needed (the same decision on every
        # rank: gen_total and A + N are global), so its generation overlaps whole steps instead of the
        # host waiting for it at the next turn
        if self.pending is not None and self.gen_total < A + N:
            self._collect()
        while self.gen_total < A + N:
            self._launch()
            self._collect()
        starts = A + np.concatenate([[0], np.cumsum(all_n)]).astype(np.int64)
        me, PS, G = c.rank, self.P * self.S, c.world
        if blocks is None:   # rank r: [starts[r], starts[r + 1]), kept at its own index
            ranges = [[(int(starts[r]), int(starts[r + 1]), int(starts[r]))] for r in range(G)]
        else:                # rank r: its blocks (j, r), global order (j, r) j-major; local order j
            nb = blocks.shape[1]
            gq = A + np.concatenate([[0], np.cumsum(blocks.T.reshape(-1))]).astype(np.int64)
            lq = np.concatenate([np.zeros((G, 1), np.int64), np.cumsum(blocks, axis=1)], axis=1)
            ranges = [[(int(gq[j * G + r]), int(gq[j * G + r + 1]), int(starts[r] + lq[r, j])) for j in range(nb)]
                      for r in range(G)]
        send = [[] for _ in range(G)]
        recv = [[] for _ in range(G)]
        def merged(rg):   # a rank's draw ranges, adjacent ones joined (one rank's blocks are one range)
            out = []
            for a, e, _ in sorted(rg):
                if e <= a:
                    continue
                if out and a <= out[-1][1]:
                    out[-1][1] = max(out[-1][1], e)
                else:
                    out.append([a, e])
            return np.asarray(out, dtype=np.int64).reshape(-1, 2)
        rarr = [merged(rg) for rg in ranges]
        for s0, cum, g, slot in self.chunks:
            for r in (range(G) if g == me else (me,)):
                js = self._subsegs_multi(s0, cum, rarr[r])
                if g == me:
                    send[r].append(slot * PS + js)
                if r == me:
                    recv[g].append(s0 + cum[js])
        cat = lambda xs: np.concatenate(xs).astype(np.int64) if xs else np.zeros(0, np.int64)
        send = [cat(x) for x in send]
        recv = [cat(x) for x in recv]
        wins = b.noise_pack(cat(send))
        if c.world > 1:
            wins = c.alltoall(wins, [len(x) for x in send], [len(x) for x in recv], what='noise windows')
        if blocks is None:
            b.noise_fill(wins, cat(recv), int(starts[me]), int(starts[me + 1]))
        else:
            b.noise_fill_ranges(wins, cat(recv), [x for x in ranges[me] if x[1] > x[0]])
        self.chunks = [ch for ch in self.chunks if ch[0] + ch[1][-1] > A + N]
        self._ahead = A + N + 4 * N   # background() launches the next round below this mark

    def background(self):
        """Next round in the background (side stream) while the steps go on; gathered when needed.
        Called once the turn's kernels are enqueued: the round's side-stream work waits for them
        (noise_shard_chunk orders it after the engine stream's pending work), so it runs beside the
        next expansion instead of the emission, select and sort."""
        if self.pending is None and self.gen_total < getattr(self, '_ahead', 0):   # >= 3 steps to generate it
            self._launch()


class DistSolve:
    """Sharded speedrun beam solve; every rank calls step() in lockstep."""

    def __init__(self, backend, comm: Comm, *, goal_pts: int, use_heuristic: bool, beam_width: int):
        self.b = backend
        self.c = comm
        self.goal = goal_pts
        self.heur = use_heuristic
        self.W = beam_width
        self.turn = 0
        self.done = False
        self.max_pts = 0
        self.winner = None                      # (turn, global rank)
        self.counts = []                        # per turn: per-rank slice sizes
        # card-set ownership of the trail (HipBackend.MIG / sb_mig.inc): parents migrate to their card-set owners
        self.mig = bool(getattr(backend, 'mig', False)) and self.c.world > 1
        # owner emission (with card-set ownership): survivors emitted on the expanding ranks, whose parents span
        # every score level, so the kept records leave every rank evenly (HipBackend.OE / sb_oe.inc)
        self.oe = self.mig and bool(getattr(backend, 'oe', False))
        # block-cyclic slices (BC): parts = blocks of the global queue, claims per part, the next beam dealt in blocks
        P = int(getattr(backend, 'parts', 0) or 0)
        self.bc = (BC and use_heuristic and bool(getattr(backend, 'goc', False)) and not self.mig and P >= 2 and
                   comm.world * P <= 64 and hasattr(backend, 'partition_blocks') and (comm.world == 1 or GKR))
        self.nb = P if self.bc else 1           # blocks per rank
        self.blocks = []                        # per turn: (world, nb) block sizes, block (r, j) = global block j * world + r
        n0 = int(backend.n_local())
        self._bounds = [0] + [n0] * self.nb     # this rank's local block bounds of the slice being expanded
        self._launch_front(1)                   # runs while the host does the turn sync / goal check (the root)
        self.lookahead = True                   # step() launches the next turn's expansion before returning
        self._front_deferred = False            # lookahead was off: the next step() launches it
        self._turn_sync()
        self.noise = ShardNoise(backend, comm) if use_heuristic else None
        self.consumed = 0                       # accepted draws used so far (global)
        self.nchunk = int(os.environ.get('SB_DIST_CHUNKS', '8'))   # key exchange / claim pipeline depth
        self.chunk_min = int(os.environ.get('SB_DIST_CHUNK_MIN', str(1 << 23)))   # fewer raw records: one chunk

    def _launch_front(self, n_global):
        """The next turn's front half, enqueued without a wait: the expansion (key-owner protocol); with card-set
        ownership the parents' owner digits and partition counts, which _turn_sync always launches itself."""
        if not self.mig:
            if self.bc:
                self.b.expand_launch(self.c.world, n_global, bounds=self._bounds)
            else:
                self.b.expand_launch(self.c.world, n_global)

    def offset(self, turn=None) -> int:
        """This rank's first parent in the rank-major numbering of turn's queue (the emission's parent numbers; with
        block-cyclic slices the receiver maps them to global ranks)."""
        cnt = self.counts[self.turn if turn is None else turn]
        return int(cnt[:self.c.rank].sum())

    def layout(self, turn):
        """(gstart, lstart) of turn's queue: gstart[r, j] = global position of rank r's block j, lstart[r] = its local
        block bounds (nb + 1).  Contiguous slices: one block per rank."""
        bs = self.blocks[turn]
        G, B = bs.shape
        gq = np.concatenate([[0], np.cumsum(bs.T.reshape(-1))]).astype(np.int64)
        gstart = gq[:-1].reshape(B, G).T
        lstart = np.concatenate([np.zeros((G, 1), np.int64), np.cumsum(bs, axis=1)], axis=1)
        return gstart, lstart

    def locate(self, turn, g):
        """(owner rank, local index) of global queue position g of turn."""
        bs = self.blocks[turn]
        G, B = bs.shape
        ends = np.cumsum(bs.T.reshape(-1))
        k = int(np.searchsorted(ends, g, side='right'))
        r, j = k % G, k // G
        gstart, lstart = self.layout(turn)
        return r, int(lstart[r, j] + g - gstart[r, j])

    def global_order(self, turn):
        """[(rank, local start, length)] runs of turn's queue in global order (tests reassemble the slices with it)."""
        bs = self.blocks[turn]
        G, B = bs.shape
        _, lstart = self.layout(turn)
        return [(r, int(lstart[r, j]), int(bs[r, j])) for j in range(B) for r in range(G)]

    # ------------------------------------------------------------ goal check (src/solver.py:438-445)
    def _turn_sync(self):
        """Once per turn, one all_gather: every rank's slice size and its first local position per
        pts value, giving the slice offsets and the global first position per pts."""
        extra = []
        if self.mig:   # enqueued first: the goal table's copy rides ahead of it (sbd_goal_table waits for that only)
            self.b.mig_launch()
        gt = self.b.goal_table().astype(np.int64)
        if self.mig:   # the slice's parents and raw children per card-set owner travel with the turn sync
            extra = self.b.mig_counts()
        elif self.bc:  # the slice's block sizes
            extra = np.diff(np.asarray(self._bounds, dtype=np.int64))
        M = self.c.allgather_array(np.concatenate([[self.b.n_local()], gt, extra]), host=True)
        if self.mig:
            W = self.c.world
            self._mig_M = M[:, 257:257 + W].copy()            # [source][owner] parents
            self._mig_R = M[:, 257 + W:257 + 2 * W].copy()    # [source][owner] their raw children
            M = M[:, :257]
        cnt = M[:, 0].copy()
        self.blocks.append(M[:, 257:257 + self.nb].copy() if self.bc else cnt[:, None].copy())
        assert (self.blocks[-1].sum(axis=1) == cnt).all(), 'block sizes disagree with the slice sizes'
        first = M[:, 1:257]
        self.counts.append(cnt)
        # the first local position per pts -> global position (its block's global start + the offset in the block)
        gstart, lstart = self.layout(len(self.blocks) - 1)
        glob = np.full(first.shape, BIG, dtype=np.int64)
        for r in range(first.shape[0]):
            ok = first[r] != NONE32
            if ok.any():
                loc = first[r][ok]
                j = np.searchsorted(lstart[r, 1:], loc, side='right')
                glob[r][ok] = gstart[r, j] + loc - lstart[r, j]
        self._goal_g = glob.min(axis=0)

    def _goal_check(self, st):
        g = self._goal_g
        win = -1
        for p in range(max(self.goal, 0), 256):
            if g[p] < BIG and (win < 0 or g[p] < win):
                win = int(g[p])
        last = -1
        while True:
            best, bp = -1, -1
            for p in range(self.max_pts + 1, 256):
                if g[p] < BIG and (best < 0 or g[p] < best):
                    best, bp = int(g[p]), p
            if best < 0 or (win >= 0 and best > win) or best <= last:
                break
            self.max_pts = bp
            st['records'].append((best, bp))
            last = best
        return win

    # ------------------------------------------------------------ one step (src/solver.py:434-457)
    def _mark(self, st, name):
        if _PHASES:
            torch.cuda.synchronize() if torch.cuda.is_available() else None
            t = time.perf_counter()
            st.setdefault('phases', {})[name] = round((t - self._t) * 1e3, 3)
            self._t = t

    def step(self) -> dict:
        c, b = self.c, self.b
        st = {'turn': self.turn, 'records': [], 'done': False}
        self._t = time.perf_counter()
        c.xbytes.clear()   # this step's exchanges (st['xbytes'], filled at its end)
        c.ncoll = c.nhost = 0
        cnt = self.counts[self.turn]
        st['n_parents'] = int(cnt.sum())
        if self.done:
            st['done'] = True
            return st
        win = self._goal_check(st)
        self._mark(st, 'goal')
        if win >= 0:
            self.done, self.winner = True, (self.turn, win)
            st.update(done=True, winner_rank=win)
            return st
        off = self.offset()
        # the expansion (launched when this slice arrived) claimed the own children; the records for the
        # other owners are partitioned by owner.  Exchange chunks: claims of chunk j overlap chunk j+1's transfer
        C = self.nchunk if st['n_parents'] * 24 >= self.chunk_min else 1
        if self._front_deferred:
            self._launch_front(st['n_parents'])
            self._front_deferred = False
        if self.mig:
            return self._dedup_mig(st, off)
        if c.world == 1 and hasattr(b, 'expand_defer') and not getattr(b, 'parts', 0):
            # one rank: no records, nothing to size, so no wait for the expansion; its raw count comes with
            # the apply's wait below
            b.expand_defer()
            b.owner_begin(0, [0])
            ret = self._ret0 if getattr(self, '_ret0', None) is not None else b.answer_buffer(0)
            self._ret0 = ret
            b.owner_finish(ret)
            self._mark(st, 'expand')
            all_n = c.gather_dev(b.apply(ret[:0])).astype(np.int64)
            st['n_raw'] = b.raw_total()
            b.apply_finish(int(all_n[0]))
            self._mark(st, 'dedup_exchange')
            return self._post_dedup(st, all_n, off)
        if getattr(b, 'parts', 0):
            return self._dedup_parts(st, off)
        cc, n_raw = b.expand_counts(C)                              # (C, world) records per chunk, owner
        M = c.allgather_array(np.concatenate([cc.ravel(), [n_raw]]))
        st['n_raw'] = int(M[:, -1].sum())
        Mc = M[:, :-1].reshape(c.world, C, c.world)                 # [source][chunk][owner]
        me = c.rank
        self._mark(st, 'expand')
        send_key = b.pack()
        self._mark(st, 'pack')
        mine = Mc[me]                                               # my records per chunk, owner
        ostart = np.concatenate([[0], np.cumsum(mine.sum(axis=0))])  # owner groups in send_key
        ochunk = np.concatenate([np.zeros((1, c.world), np.int64), np.cumsum(mine, axis=0)])
        from_src = Mc[:, :, me]                                     # [source][chunk] records to me
        src_tot = from_src.sum(axis=1)
        src_base = np.concatenate([[0], np.cumsum(src_tot)])        # global index base per source
        src_chunk = np.concatenate([np.zeros((c.world, 1), np.int64), np.cumsum(from_src, axis=1)], axis=1)
        # this rank's own children were claimed in its expansion: it has no records for itself (and at
        # world 1 there are no records and no collective at all)
        assert int(from_src[me].sum()) == 0
        handles = []
        for j in range(C):
            pieces = [send_key[int(ostart[o] + ochunk[j, o]):int(ostart[o] + ochunk[j + 1, o])]
                      for o in range(c.world)]
            if c.world > 1:
                handles.append(c.alltoall_pieces(pieces, from_src[:, j], what='records'))
            else:
                handles.append((send_key[:0], None))
        n_own = int(src_tot.sum())
        b.owner_begin(n_own, src_base[:-1])
        ret = b.answer_buffer(n_own)
        for j, (rkey, hd) in enumerate(handles):   # claims of chunk j overlap the transfer of chunk j+1
            c.wait(hd)
            if rkey.numel():
                starts = np.concatenate([[0], np.cumsum(from_src[:, j])[:-1]])
                bases = src_base[:-1] + src_chunk[:, j]
                b.owner_claim(rkey, starts, bases, ret)
        b.owner_finish(ret)
        self._mark(st, 'a2a_keys+claim')
        # answers back to the sources, one bit per answer on the wire (8x less than the answer bytes)
        own_sz = ostart[1:] - ostart[:-1]
        if c.world > 1:
            nb = lambda x: (int(x) + 7) // 8
            sp = np.concatenate([[0], np.cumsum([nb(src_tot[q]) for q in range(c.world)])])
            rp = np.concatenate([[0], np.cumsum([nb(own_sz[o]) for o in range(c.world)])])
            sbits = b.answer_buffer(int(sp[-1]))
            rbits = b.answer_buffer(int(rp[-1]))
            for q in range(c.world):
                if src_tot[q]:
                    b.pack_bits(ret[int(src_base[q]):int(src_base[q + 1])], sbits[int(sp[q]):int(sp[q + 1])])
            c.alltoall_into([sbits[int(sp[q]):int(sp[q + 1])] for q in range(c.world)],
                            [rbits[int(rp[o]):int(rp[o + 1])] for o in range(c.world)], what='answer bits')
            back = b.answer_buffer(int(ostart[-1]))
            for o in range(c.world):
                if own_sz[o]:
                    b.unpack_bits(rbits[int(rp[o]):int(rp[o + 1])], back[int(ostart[o]):int(ostart[o + 1])])
        else:
            back = ret[:0]
        all_n = c.gather_dev(b.apply(back)).astype(np.int64)   # the apply's count: one wait for both
        b.apply_finish(int(all_n[c.rank]))
        self._mark(st, 'dedup_exchange')
        return self._post_dedup(st, all_n, off)

    def _dedup_mig(self, st, off):
        """Dedup with card-set ownership (sb_mig.inc): the slice's parents go to the ranks owning their card
        sets (one all_to_all of (lo, hi, global rank) rows), which expand them with the pipelined key pass —
        takes claimed where they are generated, buys for other card-set owners exchanged as (key, tag)
        records, tags (turn, global parent rank, move) ordering like the reference's first occurrence
        (src/solver.py:446-450) — and the survivor masks come back to the slice's rank (one all_to_all), which
        goes on as in the key-owner protocol (noise, emission, joint select and rebalance unchanged)."""
        c, b = self.c, self.b
        me, W = c.rank, c.world
        M = self._mig_M
        send_sizes, recv_sizes = M[me], M[:, me]
        n_loc = int(send_sizes.sum())
        so = np.concatenate([[0], np.cumsum(send_sizes)]).astype(np.int64)
        ro = np.concatenate([[0], np.cumsum(recv_sizes)]).astype(np.int64)
        rows = b.mig_pack(off, n_loc)                      # (n_loc, 5) int32: grouped by card-set owner
        pieces = [rows[int(so[o]):int(so[o + 1])].reshape(-1) for o in range(W)]
        rflat, hd = c.alltoall_pieces(pieces, recv_sizes * 5, what='parent rows')   # 20-byte rows: 5 int32
        c.wait(hd)
        n_exp = int(ro[-1])
        b.mig_expand(rflat, n_exp, st['n_parents'])
        self._mark(st, 'migrate')
        back = self._exchange_parts(st, rec_words=3)   # 12-byte records: three int32 (key, parent rank | move)
        # survivors back to the range ranks as one bit per raw child (move order), a byte-aligned segment per
        # (expander, range rank) pair, sized by the raw counts the turn sync carried
        R = self._mig_R
        nb = lambda x: (int(x) + 7) // 8
        sb = np.concatenate([[0], np.cumsum([nb(R[q][me]) for q in range(W)])]).astype(np.int64)
        rb = np.concatenate([[0], np.cumsum([nb(R[me][o]) for o in range(W)])]).astype(np.int64)
        bits = b.bits_buffer(int(sb[-1]))
        b.mig_apply(back, bits, ro, sb[:-1], keep=self.oe)   # oe: the expand list's survivor masks kept for the emission
        rbits = b.bits_buffer(int(rb[-1]))
        c.alltoall_into([bits[int(sb[q]):int(sb[q + 1])] for q in range(W)],
                        [rbits[int(rb[o]):int(rb[o + 1])] for o in range(W)], what='survivor bits')
        all_n = c.gather_dev(b.mig_place(rbits, so, rb[:-1])).astype(np.int64)   # one wait for both
        b.apply_finish(int(all_n[c.rank]))
        self._mark(st, 'dedup_exchange')
        if self.oe:
            self._oe_emit(st, all_n, so, ro)
        return self._post_dedup(st, all_n, off)

    def _oe_emit(self, st, all_n, so, ro):
        """Owner emission: the range rank knows its parents' next_queue offsets (the survivor counts came back
        with the bits) and holds the noise draws of its range; it sends each parent's global offset and its
        survivors' draws to the rank that expanded the parent (rows' order), which emits them: scores, states,
        global parent ranks and next_queue positions (the ties' order below)."""
        c, b = self.c, self.b
        me, W = c.rank, c.world
        k_off, N = int(all_n[:me].sum()), int(all_n.sum())
        self._oe_noise(N, all_n)
        rgoff, rnoise, nb_send = b.oe_pack(k_off, N, so, int(all_n[me]))   # rows' order; noise bytes per owner
        xnb = b.oe_counts(ro)                                         # expand side: survivors per source (host)
        xgoff = b.u32_buffer(int(ro[-1]))
        c.alltoall_into([rgoff[int(so[o]):int(so[o + 1])] for o in range(W)],
                        [xgoff[int(ro[q]):int(ro[q + 1])] for q in range(W)], what='row offsets')
        xnoise = None
        if self.heur:
            ns = np.concatenate([[0], np.cumsum(nb_send)]).astype(np.int64)
            nr = np.concatenate([[0], np.cumsum(xnb)]).astype(np.int64)
            xnoise = b.byte_buffer(int(nr[-1]))
            c.alltoall_into([rnoise[int(ns[o]):int(ns[o + 1])] for o in range(W)],
                            [xnoise[int(nr[q]):int(nr[q + 1])] for q in range(W)], what='noise draws')
        b.oe_emit(xgoff, xnoise)
        self._mark(st, 'oe_emit')

    def _oe_noise(self, N, all_n):
        if self.heur:
            self.noise.prepare(self.consumed, N, all_n)
            self.consumed += N
        self._oe_noise_done = True

    def _dedup_parts(self, st, off):
        back = self._exchange_parts_goc(st) if getattr(self.b, 'goc', False) else self._exchange_parts(st)
        n_dev = self.b.apply(back)
        if self.bc:   # survivors per block (their sum is the apply's count): one wait for all
            allb = self.c.gather_dev(self.b.block_counts(self._bounds)).astype(np.int64).reshape(self.c.world, self.nb)
            self._allb = allb
            all_n = allb.sum(axis=1)
        else:
            all_n = self.c.gather_dev(n_dev).astype(np.int64)   # the apply's count: one wait for both
        self.b.apply_finish(int(all_n[self.c.rank]))
        self._mark(st, 'dedup_exchange')
        return self._post_dedup(st, all_n, off)

    def _exchange_parts_goc(self, st):
        """Dedup with the pipelined key pass and global-order claims (HipBackend.GOC, the default at world > 1 with
        key ownership).  Every part's records — this rank's own children included, as records to itself — travel
        as the parts complete (one all_to_all each, into one receive buffer, part-major), beside the later parts'
        key pass; once all have arrived, one pass claims them in virtual (source, part, record) order, which is the
        reference's (parent rank, ordinal) order (src/solver.py:446-450): first claims are then mostly the winners,
        as on one GPU, instead of being displaced by records of earlier ranks that arrive later.  Tags: turn | v.
        Then the answers go back as bits (per source and part, byte-aligned), one all_to_all."""
        c, b = self.c, self.b
        me, W, P = c.rank, c.world, b.parts
        cs = b.claim_stream()
        ctx = (lambda: torch.cuda.stream(cs)) if cs is not None else contextlib.nullcontext
        sends, recvs, handles = [], [], []
        send_base = ans_base = 0
        ret = rbuf = None
        cap = 0
        bc = self.bc
        for j in range(P):
            cnt, cap_j = b.part_counts(j)                     # waits for part j's key pass only; self included
            extra = [b.raw_total()] if j == 0 else []
            M = c.allgather_array(np.concatenate([cnt, extra]), host=True)
            if j == 0:
                st['n_raw'] = int(M[:, W].sum())
                M = M[:, :W]
                cap = cap_j
                b.owner_begin(cap, [0] * W)
                with ctx():
                    ret = getattr(b, 'ret_buffer', b.answer_buffer)(cap)
                    rbuf = b.record_buffer(cap)
                self._mark(st, 'expand')
            from_src = M[:, me]                               # records each source (this rank too) sends me
            need = ans_base + int(from_src.sum())
            if need > cap:   # the receive bound is an estimate: grow it from the exact count, contents kept
                cap = b.grow_receive(need)
                with ctx():
                    for hd in handles:                        # the earlier parts land before they are copied
                        c.wait(hd)
                    handles = []
                    g_ret, g_rec = b.answer_buffer(cap), b.record_buffer(cap)   # (new buffers: the old ones stay live
                    # in ret / rbuf until copied)
                    if ans_base:
                        g_rec[:ans_base].copy_(rbuf[:ans_base])
                        if bc:   # the earlier parts' answers (claimed already)
                            g_ret[:ans_base].copy_(ret[:ans_base])
                ret, rbuf = g_ret, g_rec
            ostart = np.concatenate([[0], np.cumsum(cnt)])
            # part j lands as [the other sources' pieces, in source order][this rank's own]: the own piece is a
            # device copy on the claim stream, not a trip through the all_to_all (RCCL copies it slowly)
            remote = from_src.copy()
            remote[me] = 0
            rtot = int(remote.sum())
            with ctx():
                key = b.part_pack(j, int(ostart[-1]), send_base)
                pieces = [key[int(ostart[o]):int(ostart[o + 1])] if o != me else key[:0] for o in range(W)]
                if W > 1:
                    _, hd = c.alltoall_pieces(pieces, remote, what='records', out=rbuf[ans_base:ans_base + rtot])
                else:    # one rank (the KP1 measurement): nothing leaves, no collective to order after
                    hd = None
                handles.append(hd)
                if cnt[me] and not bc:
                    rbuf[ans_base + rtot:need].copy_(key[int(ostart[me]):int(ostart[me + 1])])
                if bc:   # block-cyclic: part j is the global order's next range — claim it now, sources in order; this
                    # rank's own records are read where they were packed (bit 63: the send buffer), not copied
                    vs, ps, v = [], [], ans_base
                    for q in range(W):
                        vs.append(v)
                        ps.append(send_base + int(ostart[me]) - (1 << 63) if q == me else ans_base + int(remote[:q].sum()))
                        v += int(from_src[q])
                    c.wait(hd)                                # RCCL: the claim stream waits for the part's transfer
                    handles[-1] = None
                    b.owner_claim_part(j, rbuf, ans_base, need, vs, ps, ret)
            sends.append((cnt, send_base, ostart))
            recvs.append((from_src, ans_base))
            send_base += int(ostart[-1])
            ans_base = need
        # virtual order: source q's records, part by part; segment (q, j) at physical ans_base_j + the pieces of the
        # other sources before q (this rank's own piece after all of them)
        vst, pst, vseg = [], [], {}
        if bc:   # virtual order (part, source, record): every part claimed on arrival above
            for j, (fs, ab) in enumerate(recvs):
                for q in range(W):
                    vseg[(q, j)] = ab + int(fs[:q].sum())
        else:
            v = 0
            for q in range(W):
                for j, (fs, ab) in enumerate(recvs):
                    vst.append(v)
                    pst.append(ab + (int(fs.sum()) - int(fs[me]) if q == me else int(fs[:q].sum()) - (int(fs[me]) if q > me else 0)))
                    vseg[(q, j)] = v
                    v += int(fs[q])
        b.owner_total(ans_base)
        with ctx():
            if not bc:
                for hd in handles:
                    c.wait(hd)                                # RCCL: the claim stream waits for every transfer
                b.owner_claim_all(rbuf, ans_base, vst, pst, ret)
            b.owner_finish(ret)
        if cs is not None:
            torch.cuda.current_stream().wait_stream(cs)
        self._mark(st, 'a2a_keys+claim')
        nb = lambda x: (int(x) + 7) // 8
        sp = [0]
        for q in range(W):
            sp.append(sp[-1] + sum(nb(fs[q]) for fs, _ in recvs))
        rp = [0]
        for o in range(W):
            rp.append(rp[-1] + sum(nb(cn[o]) for cn, _, _ in sends))
        sbits = b.answer_buffer(sp[-1])
        rbits = b.answer_buffer(rp[-1])
        segs = []   # (answer offset, answers, bit-byte offset): every (source, part) segment in one launch
        for q in range(W):
            at = sp[q]
            for j, (fs, _) in enumerate(recvs):
                segs.append((vseg[(q, j)], int(fs[q]), at))
                at += nb(fs[q])
        b.pack_bits_segs(ret, segs, sbits)
        c.alltoall_into([sbits[sp[q]:sp[q + 1]] for q in range(W)], [rbits[rp[o]:rp[o + 1]] for o in range(W)],
                        what='answer bits')
        back = b.answer_buffer(send_base)
        segs = []
        for o in range(W):
            at = rp[o]
            for cn, sb, os_ in sends:
                segs.append((at, int(cn[o]), sb + int(os_[o])))
                at += nb(cn[o])
        b.unpack_bits_segs(rbits, segs, back)
        return back

    def _exchange_parts(self, st, rec_words=1):
        """Dedup with the pipelined key pass (b.parts exchange parts of consecutive parents): for each part,
        its records per owner (one host all_gather of the counts), its keys to their owners (all_to_all), and
        the owners' claims of them — on the claim stream, beside the next parts' key pass on the engine
        stream.  Answer indices follow arrival order (part by part, source by source), which within a source
        is (parent, ordinal) order: the claim tags (turn | source | answer index) order like the reference's
        first occurrence (src/solver.py:446-450).  Then the answers go back as bits, one all_to_all."""
        c, b = self.c, self.b
        me, W, P = c.rank, c.world, b.parts
        cs = b.claim_stream()
        ctx = (lambda: torch.cuda.stream(cs)) if cs is not None else contextlib.nullcontext
        sends, recvs = [], []
        send_base = ans_base = 0
        ret = None
        for j in range(P):
            cnt, cap = b.part_counts(j)                       # waits for part j's key pass only
            extra = [b.raw_total()] if j == 0 else []         # the raw count is known before the parts
            M = c.allgather_array(np.concatenate([cnt, extra]), host=True)
            if j == 0:
                st['n_raw'] = int(M[:, W].sum())
                M = M[:, :W]
                b.owner_begin(cap, [0] * W)
                ret = b.answer_buffer(cap)
                self._mark(st, 'expand')
            from_src = M[:, me]                               # records each source sends me in this part
            if ans_base + int(from_src.sum()) > cap:
                # the receive bound is an estimate (max raw ratio so far + 50%), not a worst case; the exact count
                # is known here, before the part's claims: grow the lost bits / tags and the answer buffer
                cap = b.grow_receive(ans_base + int(from_src.sum()))
                with ctx():
                    grown = b.answer_buffer(cap)
                    if ans_base:
                        grown[:ans_base].copy_(ret[:ans_base])
                ret = grown
            ostart = np.concatenate([[0], np.cumsum(cnt)])
            with ctx():
                key = b.part_pack(j, int(ostart[-1]), send_base)
                rw = rec_words
                pieces = [key[rw * int(ostart[o]):rw * int(ostart[o + 1])] for o in range(W)]
                rkey, hd = c.alltoall_pieces(pieces, from_src * rw, what='records')
                c.wait(hd)                                    # RCCL: the claim stream waits for the transfer
                if rkey.numel() and rw == 3:                  # (key, tag) records: tags carry the global order
                    b.mig_claim(rkey, ans_base, ret)
                elif rkey.numel():
                    starts = np.concatenate([[0], np.cumsum(from_src)[:-1]])
                    b.owner_claim(rkey, starts, ans_base + starts, ret)
            sends.append((cnt, send_base, ostart))
            recvs.append((from_src, ans_base))
            send_base += int(ostart[-1])
            ans_base += int(from_src.sum())
        b.owner_total(ans_base)
        with ctx():
            b.owner_finish(ret)
        if cs is not None:
            torch.cuda.current_stream().wait_stream(cs)
        self._mark(st, 'a2a_keys+claim')
        # answers back to the sources as bits: to source q, its (part j) segments in part order
        nb = lambda x: (int(x) + 7) // 8
        sp = [0]
        for q in range(W):
            sp.append(sp[-1] + sum(nb(fs[q]) for fs, _ in recvs))
        rp = [0]
        for o in range(W):
            rp.append(rp[-1] + sum(nb(cn[o]) for cn, _, _ in sends))
        sbits = b.answer_buffer(sp[-1])
        rbits = b.answer_buffer(rp[-1])
        segs = []   # (answer offset, answers, bit-byte offset): every (source, part) segment in one launch
        for q in range(W):
            at = sp[q]
            for fs, ab in recvs:
                segs.append((ab + int(np.sum(fs[:q])), int(fs[q]), at))
                at += nb(fs[q])
        b.pack_bits_segs(ret, segs, sbits)
        c.alltoall_into([sbits[sp[q]:sp[q + 1]] for q in range(W)], [rbits[rp[o]:rp[o + 1]] for o in range(W)],
                        what='answer bits')
        back = b.answer_buffer(send_base)
        segs = []
        for o in range(W):
            at = rp[o]
            for cn, sb, os_ in sends:
                segs.append((at, int(cn[o]), sb + int(os_[o])))
                at += nb(cn[o])
        b.unpack_bits_segs(rbits, segs, back)
        return back

    def _post_dedup(self, st, all_n, off):
        """noise, emission, joint select, rebalance and receive of a step (after the dedup exchange)."""
        c, b = self.c, self.b
        k_off = int(all_n[:c.rank].sum())
        N = int(all_n.sum())
        st['n_unique'] = N
        if N == 0:   # queue empties: `puzzle` is the last parent (src/solver.py:438,459)
            last = st['n_parents'] - 1
            self.done, self.winner = True, (self.turn, last)
            st.update(done=True, winner_rank=last)
            return st
        oe = getattr(self, '_oe_noise_done', False)
        self._oe_noise_done = False
        if not oe:   # (owner emission: the range ranks' draws went out with the offsets, _oe_emit)
            if self.heur:
                self.noise.prepare(self.consumed, N, all_n, self._allb if self.bc else None)
                self.consumed += N
            self._mark(st, 'noise')
            b.emit(k_off, N, off)
            self._mark(st, 'emit')
        K = min(N, self.W) if self.heur else N
        G = c.world
        if self.heur:
            has_top = N > self.W
            nsp = G * self.nb   # destination ranges: the ranks, or (block-cyclic) the next beam's world x parts blocks
            if self.bc and P0 != 1.0 and self.nb > 1:   # part 0's blocks P0 times the others': its key pass, which the
                # claims wait for, is shorter (any boundaries are valid, the same on every rank)
                wt = np.where(np.arange(nsp) < G, P0, 1.0)
                cw = np.cumsum(wt)[:-1] / wt.sum()
                pos = ([self.W] if has_top else []) + [max(1, int(np.ceil(K * x))) for x in cw]
            else:
                pos = ([self.W] if has_top else []) + [max(1, -(-j * K // nsp)) for j in range(1, nsp)]
            eq_all = None
            if pos:
                # block-cyclic: the block boundaries stop refining once their bucket holds <= 1/16 of a block
                approx = (int(has_top), max(1, K // (nsp * 16))) if self.bc else None
                self._multiselect(pos, st, approx)
                self._mark(st, 'sel_passes')
                if has_top and oe:   # ties at the keep boundary in next_queue order: by position, over all ranks
                    tp, need = b.oe_ties()
                    allt = c.allgather_var(tp)
                    pstar = int(np.partition(allt, need - 1)[need - 1]) if need > 0 else -1
                elif has_top and self.bc:   # ties per block: kept in global (block, rank) order
                    eq_all = c.allgather_tensor(b.sel_eq_blocks(self._qstart())).reshape(-1)
                elif has_top:
                    eq_all = c.allgather_tensor(b.sel_eq()).reshape(-1)
            self._mark(st, 'sel_eq')
            if oe:
                dest_dev = b.oe_partition(has_top, pstar if has_top else -1, len(pos) - int(has_top), G)
            elif self.bc:
                dest_dev = b.partition_blocks(has_top, eq_all, c.rank, G, self.nb, qstart=self._qstart())
            else:
                dest_dev = b.partition(has_top, eq_all, c.rank, len(pos) - int(has_top), G)
        elif oe:
            dest_dev = b.oe_partition_bfs(N, G)
        else:
            dest_dev = b.partition_bfs(k_off, N, G)
        self._mark(st, 'select')
        # 20-byte kept records when every global parent rank of the turn fits 25 bits (the same choice on every rank);
        # world > 1 with key ownership: grouped by (parent, destination) on the wire (sbd_pack_kept_grouped)
        rec20 = st['n_parents'] <= (1 << 25)
        if self.bc and c.world > 1:
            assert rec20, 'block-cyclic slices need global parent ranks below 2^25 (20-byte records)'
            self._rebalance_grouped_bc(st, all_n)
        elif GKR and c.world > 1 and rec20 and not oe and not self.mig and hasattr(b, 'pack_kept_grouped'):
            self._rebalance_grouped(st, all_n)
        else:
            self._rebalance(st, all_n, K, dest_dev, oe, rec20)
        if self.heur:
            self.noise.background()
        if getattr(b, 'timing', False):   # device time of this step's key kernels (the bench's world > 1 roofline), read
            st['keypass_ms'] = b.keypass_ms()   # here, long done, not on the way from the apply to the emission
        if self.lookahead:
            self._launch_front(K)   # the next turn's expansion (K parents in all) overlaps its goal check
        else:   # a benchmark's window edge (bench.py): the next step() launches it
            self._front_deferred = True
        self._turn_sync()
        self._mark(st, 'rebalance')
        st['xbytes'] = dict(c.xbytes)
        st['collectives'] = (c.ncoll, c.nhost)   # (device-group rounds, host metadata rounds) of this step
        self.turn += 1
        st['n_kept'] = int(self.counts[-1].sum())
        return st

    def _rebalance_grouped(self, st, all_n):
        """kept records to their destination ranges as (parent, destination) groups: one count exchange of
        (children, groups) pairs, one all_to_all of the segments (5 G + ceil(C / 2) u32 each; this rank's own
        copied), the receiver expands them into the 20-byte records, then receives them as usual."""
        c, b = self.c, self.b
        buf, cnt2 = b.pack_kept_grouped(all_n[c.rank])   # ahead of the counts
        send2, recv2 = c.alltoall_counts_dev(cnt2)
        send2 = np.asarray(send2, dtype=np.int64).reshape(c.world, 2)
        recv2 = np.asarray(recv2, dtype=np.int64).reshape(c.world, 2)
        ssz = 5 * send2[:, 1] + (send2[:, 0] + 1) // 2
        rsz = 5 * recv2[:, 1] + (recv2[:, 0] + 1) // 2
        self._mark(st, 'pack_kept')
        me = c.rank
        so = np.concatenate([[0], np.cumsum(ssz)]).astype(np.int64)
        ro = np.concatenate([[0], np.cumsum(rsz)]).astype(np.int64)
        rbuf = torch.empty(max(int(ro[-1]), 1), dtype=torch.int32, device=buf.device)
        pieces = [buf[int(so[q]):int(so[q + 1])] if q != me else buf[:0] for q in range(c.world)]
        outs = [rbuf[int(ro[q]):int(ro[q + 1])] if q != me else rbuf[:0] for q in range(c.world)]
        c.alltoall_into(pieces, outs, what='kept records')
        rbuf[int(ro[me]):int(ro[me + 1])].copy_(buf[int(so[me]):int(so[me + 1])])
        self._mark(st, 'a2a_kept')
        rrec = b.unpack_kept(rbuf, ro[:-1], recv2[:, 1], recv2[:, 0])
        b.receive(rrec, self.heur)

    def _qstart(self):
        """This rank's blocks' first local next_queue positions (nb + 1)."""
        return np.concatenate([[0], np.cumsum(self._allb[self.c.rank])]).astype(np.int64)

    def _rebalance_grouped_bc(self, st, all_n):
        """Block-cyclic slices: the kept records go to the next beam's blocks as (parent, destination block) groups.
        One count exchange carries, per destination rank, its blocks' (children, groups) and the children per (source
        block, destination block); one all_to_all moves the segments; the receiver expands them in (its block, source
        block, source) order — the global next_queue order within each block, which the stable score sort keeps for ties
        (a score's ties never span two blocks) — with the senders' parent numbers mapped to global ranks."""
        c, b = self.c, self.b
        G, nb, me = c.world, self.nb, c.rank
        D = G * nb
        buf, cnt2 = b.pack_kept_grouped(all_n[me], ndig=D)            # (children, groups) per digit (rank, block)
        sub = b.dest_subcounts(self._qstart(), D)                       # (nb source blocks, D digits)
        send = torch.cat([cnt2.reshape(G, 2 * nb), sub.reshape(nb, G, nb).permute(1, 0, 2).reshape(G, nb * nb)], dim=1)
        send2, recv2 = c.alltoall_counts_dev(send.contiguous())
        send2 = np.asarray(send2, dtype=np.int64).reshape(G, 2 * nb + nb * nb)
        recv2 = np.asarray(recv2, dtype=np.int64).reshape(G, 2 * nb + nb * nb)
        sch, sgr = send2[:, 0:2 * nb:2], send2[:, 1:2 * nb:2]           # (dest rank, its block)
        rch, rgr = recv2[:, 0:2 * nb:2], recv2[:, 1:2 * nb:2]           # (source, my block)
        rsub = recv2[:, 2 * nb:].reshape(G, nb, nb)                      # (source, source block, my block)
        ssz = (5 * sgr + (sch + 1) // 2).sum(axis=1)
        rseg = 5 * rgr + (rch + 1) // 2                                  # u32 per (source, my block) segment
        rsz = rseg.sum(axis=1)
        self._mark(st, 'pack_kept')
        so = np.concatenate([[0], np.cumsum(ssz)]).astype(np.int64)
        ro = np.concatenate([[0], np.cumsum(rsz)]).astype(np.int64)
        rbuf = torch.empty(max(int(ro[-1]), 1), dtype=torch.int32, device=buf.device)
        pieces = [buf[int(so[q]):int(so[q + 1])] if q != me else buf[:0] for q in range(G)]
        outs = [rbuf[int(ro[q]):int(ro[q + 1])] if q != me else rbuf[:0] for q in range(G)]
        c.alltoall_into(pieces, outs, what='kept records')
        rbuf[int(ro[me]):int(ro[me + 1])].copy_(buf[int(so[me]):int(so[me + 1])])
        self._mark(st, 'a2a_kept')
        # segments (source q, my block p), source-major; children concatenated in that order
        bases = ro[:-1, None] + np.concatenate([np.zeros((G, 1), np.int64), np.cumsum(rseg, axis=1)[:, :-1]], axis=1)
        # target order (my block p, source block j, source q): run starts
        cnt_pjq = rsub.transpose(2, 1, 0)                                # (p, j, q)
        dst0 = np.concatenate([[0], np.cumsum(cnt_pjq.reshape(-1))])[:-1].reshape(nb, nb, G)
        perm, src = [], 0   # (non-empty runs only: an empty run would share its start with the next one)
        for q in range(G):
            for p in range(nb):
                for j in range(nb):
                    if rsub[q, j, p]:
                        perm.append((src, int(dst0[p, j, q])))
                    src += int(rsub[q, j, p])
        # the senders' parent numbers (rank-major over this turn's slices) -> global ranks, non-empty blocks
        gstart, lstart = self.layout(self.turn)
        voff = np.concatenate([[0], np.cumsum(self.counts[self.turn])])
        bs = self.blocks[self.turn]
        pmap = sorted((int(voff[r] + lstart[r, j]), int(gstart[r, j])) for r in range(G) for j in range(nb) if bs[r, j])
        rrec = b.unpack_kept(rbuf, bases.reshape(-1), rgr.reshape(-1), rch.reshape(-1), perm=perm, pmap=pmap)
        b.receive(rrec, self.heur)
        self._bounds = [0] + np.cumsum(rch.sum(axis=0)).astype(np.int64).tolist()

    def _rebalance(self, st, all_n, K, dest_dev, oe, rec20):
        c, b = self.c, self.b
        rec = b.pack_kept(b.oe_n() if oe else all_n[c.rank], rec20=rec20)   # ahead of the counts
        if c.world == 1 and self.bc:   # every kept record stays; its blocks' sizes are the next parts' bounds
            dest_counts = dest_dev.cpu().numpy().astype(np.int64)
            self._bounds = [0] + np.cumsum(dest_counts).tolist()
            dest_counts = recv = np.array([int(dest_counts.sum())], dtype=np.int64)
        elif c.world == 1:   # every kept record stays: K of them, known here (no round trip)
            dest_counts = recv = np.array([K], dtype=np.int64)
        else:
            dest_counts, recv = c.alltoall_counts_dev(dest_dev)
        self._mark(st, 'pack_kept')
        if c.world > 1:   # records arrive source rank by source rank; this rank's own are copied
            me = c.rank
            so = np.concatenate([[0], np.cumsum(dest_counts)]).astype(np.int64)
            ro = np.concatenate([[0], np.cumsum(recv)]).astype(np.int64)
            rrec = torch.empty((int(ro[-1]),) + tuple(rec.shape[1:]), dtype=rec.dtype, device=rec.device)
            pieces = [rec[int(so[q]):int(so[q + 1])] if q != me else rec[:0] for q in range(c.world)]
            outs = [rrec[int(ro[q]):int(ro[q + 1])] if q != me else rrec[:0] for q in range(c.world)]
            c.alltoall_into(pieces, outs, what='kept records')
            rrec[int(ro[me]):int(ro[me + 1])].copy_(rec[int(so[me]):int(so[me + 1])])
        else:
            rrec = rec[:int(dest_counts.sum())]
            ro = np.array([0, rrec.shape[0]], dtype=np.int64)
        self._mark(st, 'a2a_kept')
        if oe:   # each source's records in position order: the receive merges them
            b.oe_segments(ro)
        b.receive(rrec, self.heur)

    SEL_PASSES = 7   # ceil(64 / 10): passes after the last digit are no-ops on the device

    def _multiselect(self, positions, st=None, approx=None):
        """Global key at each 1-based position of the (score desc) order and how many of its ties
        precede the position, left in the backend's select state: MSB radix select over 10-bit
        digits below the bits common to every key (all_reduce(MIN) of the encoded range); per pass
        a histogram per distinct prefix, all_reduce(SUM) on the device, a pick kernel; after the
        first pass each rank keeps only its keys in the chosen buckets.  Nothing here waits on the
        host: the passes and collectives are enqueued on the engine's stream."""
        c, b = self.c, self.b
        rng = b.key_range()
        c.allreduce_tensor(rng, dist.ReduceOp.MIN)
        if approx is not None:   # (positions approx[0].. are block boundaries, frozen at <= approx[1] keys a bucket)
            b.sel_begin_approx(positions, rng, *approx)
        else:
            b.sel_begin(positions, rng)
        src = 0
        for p in range(self.SEL_PASSES + (len(positions) > 16)):   # 8-bit digits once more than 16 prefixes are live
            h = b.sel_hist(src)
            c.allreduce_tensor(h)
            b.sel_pick(h)
            if p == 0:
                b.sel_compact()
                src = 1

    def run(self, max_turns=10_000):
        trace = []
        while not self.done and len(trace) < max_turns:
            trace.append(self.step())
        return trace

    def path(self):
        """Root..winner states (src/solver.py:459-464); identical on every rank."""
        t, r = self.winner
        out = []
        while t >= 0:
            owner, loc = self.locate(t, r)
            vals = [0, 0, 0]
            if owner == self.c.rank:
                lo, hi, par = self.b.turn_state(t, loc)
                vals = [_u64_to_i64(lo), _u64_to_i64(hi), par]
            lo, hi, par = self.c.broadcast_ints(vals, owner)
            out.append((lo & 0xFFFFFFFFFFFFFFFF, hi & 0xFFFFFFFFFFFFFFFF))
            r = par
            t -= 1
        return out[::-1]


class SerializedBackend:
    """Profiling aid (bench_dist.py with SB_DIST_SERIALIZE=1): several ranks sharing one GPU run their
    backend calls under one inter-process lock (flock on `lock_path`), each call synchronised before the
    lock is released, so a kernel trace shows every rank's kernels alone on the device — the device time
    one rank's own GPU would spend.  Ranks may make different calls (e.g. pack_bits only for non-empty
    segments): the lock needs no matching call counts.  Results are unchanged."""

    def __init__(self, backend, lock_path=None):
        import tempfile
        self._b = backend
        path = lock_path or os.path.join(tempfile.gettempdir(),
                                         f'sb_serial_{os.environ.get("MASTER_PORT", "0")}.lock')
        self._fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o600)

    def lock(self):
        """The inter-process device lock as a context manager (Comm.devlock: gloo's staging copies)."""
        import contextlib
        import fcntl

        @contextlib.contextmanager
        def held():
            fcntl.flock(self._fd, fcntl.LOCK_EX)
            try:
                yield
            finally:
                fcntl.flock(self._fd, fcntl.LOCK_UN)
        return held()

    def __getattr__(self, name):
        attr = getattr(self._b, name)
        if not callable(attr):
            return attr

        def call(*a, **k):
            with self.lock():
                out = attr(*a, **k)
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
            return out
        return call


class TimedProxy:
    """Profiling aid (bench_dist.py with SB_DIST_HOSTPROF=1): host time spent inside each method of the
    wrapped backend / Comm (calls that wait for the device show their wait here); the step's wall time
    minus the sum is the Python orchestration between calls."""

    def __init__(self, obj, table):
        self._o, self._t = obj, table

    def __getattr__(self, name):
        attr = getattr(self._o, name)
        if not callable(attr):
            return attr

        def call(*a, **k):
            t0 = time.perf_counter()
            out = attr(*a, **k)
            e = self._t.setdefault(name, [0, 0.0])
            e[0] += 1
            e[1] += time.perf_counter() - t0
            return out
        return call


class _DevArray:
    """Engine-owned device memory as a torch tensor (__cuda_array_interface__, no copy): the packed records the
    expansion wrote, sent by the all_to_all straight from where they are."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {'shape': (int(n),), 'typestr': '<i8', 'data': (int(ptr or 0), False),
                                         'version': 2, 'strides': None}


class HipBackend:
    """Per-rank primitives on the MI355X engine (libsplendor_beam.so, sbd_* entry points).

    Exchange buffers are torch tensors on this rank's device, handed to the engine by device
    pointer.  The engine runs on torch's current stream (sbd_set_stream), the stream the
    collectives use, so kernels and exchanges are ordered on the device; the host waits only where
    it needs a value (counts that size an all_to_all, the goal table).
    """

    # world > 1: the key pass (flags bit 6, sb_keypass.inc) instead of the expansion kernel + owner partition
    KEYPASS = os.environ.get('SB_DIST_KEYPASS', '1') != '0'
    # world > 1: card-set ownership of the trail (flags bit 8, sb_mig.inc) instead of key ownership.  NOT bit-exact
    # by construction: the reference's equality is the 64-bit key (src/solver.py:332-336), and two states of
    # different card sets with an equal key are claimed on two owners and both kept (≈0.06 such pairs expected
    # per C5 solve, none in any golden).  Opt-in only; every surface that enables it says so (MIG_CAVEAT).
    MIG = os.environ.get('SB_DIST_MIG', '0') == '1'
    MIG_CAVEAT = ('card-set ownership of the trail (SB_DIST_MIG=1 / flags bit 8) is not bit-exact by construction: '
                  'two states of different card sets with an equal 64-bit key are both kept, where the reference '
                  '(hash equality, src/solver.py:332-336) keeps the first')
    # with card-set ownership: owner emission (flags bit 9, sb_oe.inc), survivors emitted on the expanding ranks
    OE = os.environ.get('SB_DIST_OE', '0') == '1'
    PARTS = int(os.environ.get('SB_DIST_PARTS', '4'))   # exchange parts of the pipelined key pass (<= 16)
    # key ownership, world > 1: global-order claims (flags bit 11, sb_dist.inc k_claim_goc): own children become
    # records to this rank and all records are claimed in one pass in global order once every part has arrived
    GOC = os.environ.get('SB_DIST_GOC', '1') != '0'
    # measurement aid: the world > 1 key-owner path (pipelined key pass, global-order claims) at world 1, so one
    # GPU runs a rank's whole sharded device work with its streams overlapping as on an 8-GPU node (no exchange)
    KP1 = os.environ.get('SB_DIST_KP1') == '1'
    PRIO = os.environ.get('SB_DIST_PRIO', '1') == '1'   # A/B (profiles/r6/s6): world-1 key-pass run 8.04-8.09 -> 7.86-7.93 ms

    def __init__(self, *, rank: int, world: int, device_index: int, goal_pts: int, use_heuristic: bool,
                 heuristic: int, beam_width: int, mt_state625, root=(0, 0), visited_log2: int = 0,
                 extra_flags: int = 0):
        import ctypes as C
        from . import _lib as L
        self.C, self.L = C, L
        L.ensure_tables()
        self.lib = L.lib()
        self._bind()
        self.device = torch.device('cuda', device_index)
        torch.cuda.set_device(self.device)
        self.mig = bool(self.MIG or (int(extra_flags) & 256)) and world > 1
        self.oe = self.mig and bool(self.OE or (int(extra_flags) & 512))
        if self.mig and rank == 0:
            import warnings
            warnings.warn(self.MIG_CAVEAT, stacklevel=2)
        self.timing = bool(int(extra_flags) & 1)   # key-pass device time per step (sbd_keypass_ms)
        xw = world > 1 or (self.KP1 and not self.mig)   # the world > 1 key-owner machinery (KP1: at world 1 too)
        self.goc = bool(self.GOC or (world == 1 and self.KP1)) and self.KEYPASS and xw and not self.mig
        self.heur = bool(use_heuristic)
        cfg = L.SbConfig(goal_pts=int(goal_pts), use_heuristic=int(bool(use_heuristic)), heuristic=int(heuristic),
                         device=int(device_index), beam_width=int(beam_width), visited_log2=int(visited_log2),
                         flags=2 | (int(extra_flags) & 1201) | (64 if self.KEYPASS and xw else 0) |
                         (256 if self.mig else 0) | (512 if self.oe else 0) | (2048 if self.goc else 0),
                         world_size=int(world), rank=int(rank))
        h = C.c_void_p()
        st = np.ascontiguousarray(np.array(mt_state625, dtype=np.uint32))
        L.check(self.lib.sb_create(C.byref(cfg), st, int(root[0]), int(root[1]), C.byref(h)), 'sb_create')
        self.h = h
        self.world = world
        # one stream for the engine's kernels and the collectives: ordered without host syncs
        # SB_DIST_PRIO=1: the engine stream (key passes, packs, the step's short kernels) at high priority over the claim
        # stream, whose persistent claim grid would otherwise hold back the engine's single-workgroup scans
        self.stream = torch.cuda.Stream(self.device, priority=-1 if self.PRIO else 0)
        torch.cuda.set_stream(self.stream)
        L.check(self.lib.sbd_set_stream(self.h, C.c_void_p(self.stream.cuda_stream)), 'sbd_set_stream')
        # world > 1: the pipelined key pass; received records are claimed on a second stream beside it
        self.parts = max(1, min(16, self.PARTS)) if ((self.KEYPASS or self.mig) and xw) else 0
        self.cstream = None
        if self.parts:
            self.cstream = torch.cuda.Stream(self.device)
            L.check(self.lib.sbd_set_claim_stream(self.h, C.c_void_p(self.cstream.cuda_stream)), 'sbd_set_claim_stream')

    def _bind(self):
        C, lib = self.C, self.lib
        if getattr(lib, '_sbd_bound', False):
            return
        vp, i64, u64, i32 = C.c_void_p, C.c_int64, C.c_uint64, C.c_int32
        p64 = C.POINTER(C.c_int64)
        lib.sbd_goal_table.argtypes = [vp, vp]
        lib.sbd_expand_launch.argtypes = [vp, i32]
        lib.sbd_expand_counts.argtypes = [vp, i32, vp, p64]
        lib.sbd_expand_parts.argtypes = [vp, i32, i32, i64, vp]
        lib.sbd_part_counts.argtypes = [vp, i32, vp, p64]
        lib.sbd_part_pack.argtypes = [vp, i32, vp, i64]
        lib.sbd_send_buffer.argtypes = [vp, vp, p64]
        lib.sbd_set_claim_stream.argtypes = [vp, vp]
        lib.sbd_owner_total.argtypes = [vp, i64]
        lib.sbd_grow_receive.argtypes = [vp, i64, p64]
        lib.sbd_expand_defer.argtypes = [vp]
        lib.sbd_raw_total.argtypes = [vp, p64]
        lib.sbd_pack.argtypes = [vp, vp, vp]
        lib.sbd_owner_begin.argtypes = [vp, i64, i32, vp]
        lib.sbd_owner_claim.argtypes = [vp, vp, i64, i32, vp, vp, vp]
        lib.sbd_owner_finish.argtypes = [vp, vp]
        lib.sbd_owner_claim_all.argtypes = [vp, vp, i64, i32, vp, vp, vp]
        lib.sbd_owner_claim_part.argtypes = [vp, i32, vp, i64, i64, i32, vp, vp, vp]
        lib.sbd_block_counts.argtypes = [vp, i32, vp, vp]
        lib.sbd_sel_eq_blocks.argtypes = [vp, i32, vp, vp]
        lib.sbd_partition_blocks.argtypes = [vp, i32, vp, i32, i32, i32, vp, vp, vp]
        lib.sbd_dest_subcounts.argtypes = [vp, i32, vp, i32, vp]
        lib.sbd_noise_fill_ranges.argtypes = [vp, i32, vp, vp, i32, vp, vp, vp]
        lib.sbd_pack_bits.argtypes = [vp, vp, i64, vp]
        lib.sbd_unpack_bits.argtypes = [vp, vp, i64, vp]
        lib.sbd_pack_bits_segs.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        lib.sbd_unpack_bits_segs.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        lib.sbd_apply.argtypes = [vp, vp, vp]
        lib.sbd_apply_finish.argtypes = [vp, i64]
        lib.sbd_emit.argtypes = [vp, u64, u64, i64]
        lib.sbd_key_range.argtypes = [vp, vp]
        lib.sbd_sel_begin.argtypes = [vp, i32, vp, vp]
        lib.sbd_sel_begin_approx.argtypes = [vp, i32, vp, vp, i32, i64]
        lib.sbd_sel_hist.argtypes = [vp, i32, vp]
        lib.sbd_sel_pick.argtypes = [vp, vp]
        lib.sbd_sel_compact.argtypes = [vp]
        lib.sbd_sel_eq.argtypes = [vp, vp]
        lib.sbd_set_stream.argtypes = [vp, vp]
        lib.sbd_noise_info.argtypes = [vp, vp]
        lib.sbd_noise_chunk.argtypes = [vp, i32, vp]
        lib.sbd_noise_sync.argtypes = [vp]
        lib.sbd_noise_pack.argtypes = [vp, i32, vp, vp]
        lib.sbd_noise_fill.argtypes = [vp, i32, vp, vp, u64, u64]
        lib.sbd_partition.argtypes = [vp, i32, vp, i32, i32, i32, vp]
        lib.sbd_partition_bfs.argtypes = [vp, u64, u64, i32, vp]
        lib.sbd_pack_kept.argtypes = [vp, vp, i32]
        lib.sbd_pack_kept_grouped.argtypes = [vp, vp, i64, vp]
        lib.sbd_unpack_kept.argtypes = [vp, vp, i32, p64, p64, p64, vp, i32, vp, i32, vp]
        lib.sbd_receive.argtypes = [vp, vp, i64, i32]
        lib.sbd_mark_done.argtypes = [vp, i64]
        lib.sbd_mig_launch.argtypes = [vp, i32]
        lib.sbd_mig_counts.argtypes = [vp, vp]
        lib.sbd_mig_pack.argtypes = [vp, i64, vp]
        lib.sbd_mig_expand.argtypes = [vp, i32, i32, i64, vp, i64]
        lib.sbd_mig_claim.argtypes = [vp, vp, i64, i64, vp]
        lib.sbd_mig_apply.argtypes = [vp, vp, vp, i32, vp, vp]
        lib.sbd_mig_place.argtypes = [vp, vp, i32, vp, vp, vp]
        lib.sbd_keypass_ms.argtypes = [vp, vp]
        lib.sbd_oe_pack.argtypes = [vp, u64, u64, vp, vp, i32, vp, vp]
        lib.sbd_oe_counts.argtypes = [vp, i32, vp, vp]
        lib.sbd_oe_emit.argtypes = [vp, vp, vp]
        lib.sbd_oe_ties.argtypes = [vp, vp, vp]
        lib.sbd_oe_tie_read.argtypes = [vp, vp, i64]
        lib.sbd_oe_partition.argtypes = [vp, i32, i64, i32, i32, vp]
        lib.sbd_oe_partition_bfs.argtypes = [vp, u64, i32, vp]
        lib.sbd_oe_segments.argtypes = [vp, i32, vp]
        lib._sbd_bound = True

    def _chk(self, rc, what):
        self.L.check(rc, what)

    def _sync(self):
        torch.cuda.synchronize(self.device)

    def close(self):
        self._rbuf = self._abuf = self._send_t = None   # (the turn buffers kept across turns)
        if getattr(self, 'h', None):
            self.lib.sb_destroy(self.h)
            self.h = None

    # ---------------------------------------------------------------- queries
    def n_local(self) -> int:
        C = self.C
        nt = C.c_int32()
        self._chk(self.lib.sb_num_turns(self.h, C.byref(nt)), 'sb_num_turns')
        n = C.c_int64()
        self._chk(self.lib.sb_turn_size(self.h, nt.value - 1, C.byref(n)), 'sb_turn_size')
        return n.value

    def goal_table(self) -> np.ndarray:
        out = np.zeros(256, np.uint32)
        self._chk(self.lib.sbd_goal_table(self.h, out.ctypes.data), 'sbd_goal_table')
        return out

    def turn_state(self, t: int, r: int):
        lo = np.zeros(1, np.uint64)
        hi = np.zeros(1, np.uint64)
        par = np.zeros(1, np.uint32)
        self._chk(self.lib.sb_read_turn(self.h, t, r, 1, lo.ctypes.data, hi.ctypes.data, par.ctypes.data, None),
                  'sb_read_turn')
        return int(lo[0]), int(hi[0]), int(par[0])

    def turn_keys(self, t: int) -> np.ndarray:
        """State keys of this rank's slice of turn t (the slice in global queue order)."""
        C = self.C
        n = C.c_int64()
        self._chk(self.lib.sb_turn_size(self.h, int(t), C.byref(n)), 'sb_turn_size')
        key = np.zeros(n.value, np.uint64)
        if n.value:
            self._chk(self.lib.sb_read_turn(self.h, int(t), 0, n.value, None, None, None, key.ctypes.data),
                      'sb_read_turn')
        return key

    def mt_state(self) -> np.ndarray:
        out = np.zeros(625, np.uint32)
        self._chk(self.lib.sb_get_mt_state(self.h, out), 'sb_get_mt_state')
        return out

    def visited_capacity(self) -> tuple[int, int]:
        """(slots, rebuilds) of this rank's owner shard of the visited set."""
        return self.L.visited_capacity(self.h)

    def visited_stats(self) -> dict:
        """Growth record of this rank's owner shard (sb_visited_stats)."""
        return self.L.visited_stats(self.h)

    # ---------------------------------------------------------------- step primitives
    def expand_launch(self, world, n_global=0, bounds=None):
        """Enqueue this turn's expansion (own children claimed, records for the other owners); no wait.
        world > 1: the pipelined key pass in self.parts exchange parts (n_global: the turn's parents over
        all ranks, bounds what this rank receives; bounds: the parts' local parent bounds, block-cyclic slices)."""
        self.world_x = int(world)
        if self.parts and (world > 1 or self.KP1):
            bd = None
            if bounds is not None:
                bd = np.ascontiguousarray(np.asarray(bounds, dtype=np.int64))
                assert len(bd) == self.parts + 1
            self._chk(self.lib.sbd_expand_parts(self.h, int(world), int(self.parts), int(n_global),
                                                bd.ctypes.data if bd is not None else None), 'sbd_expand_parts')
            return
        self._chk(self.lib.sbd_expand_launch(self.h, int(world)), 'sbd_expand_launch')

    def claim_stream(self):
        return self.cstream

    def part_counts(self, j):
        """Part j's records per owner (waits for its key pass) and the turn's receive bound."""
        C = self.C
        cnt = np.zeros(self.world_x, np.int64)
        cap = C.c_int64()
        self._chk(self.lib.sbd_part_counts(self.h, int(j), cnt.ctypes.data, C.byref(cap)), 'sbd_part_counts')
        return cnt, cap.value

    def part_pack(self, j, n, send_base):
        """Part j's n records in owner groups (on the claim stream: the caller's current stream); with card-set
        ownership each record is 12 bytes (key, global parent rank << 7 | move), 3n int32.  Global-order claims: packed
        by the expansion itself into the engine's send buffer — a view of it at send_base."""
        if self.goc:
            self._chk(self.lib.sbd_part_pack(self.h, int(j), None, int(send_base)), 'sbd_part_pack')
            if j == 0 or getattr(self, '_send_t', None) is None:
                ptr, cap = self.C.c_void_p(), self.C.c_int64()
                self._chk(self.lib.sbd_send_buffer(self.h, self.C.byref(ptr), self.C.byref(cap)), 'sbd_send_buffer')
                self._send_t = torch.as_tensor(_DevArray(ptr.value, cap.value), device=self.device)
            return self._send_t[int(send_base):int(send_base) + int(n)]
        if self.mig:   # 12-byte records, three int32 each
            key = self._empty(max(3 * int(n), 1), torch.int32)[:3 * int(n)]
        else:
            key = self._empty(max(int(n), 1))[:int(n)]
        self._chk(self.lib.sbd_part_pack(self.h, int(j), key.data_ptr() if n else None, int(send_base)), 'sbd_part_pack')
        return key

    def grow_receive(self, n_needed) -> int:
        """The turn's receive bound raised to >= n_needed (sbd_grow_receive: drains this rank's streams, keeps the
        lost bits / tags so far); returns the new bound."""
        cap = self.C.c_int64()
        self._chk(self.lib.sbd_grow_receive(self.h, int(n_needed), self.C.byref(cap)), 'sbd_grow_receive')
        return cap.value

    def owner_total(self, n):
        self._chk(self.lib.sbd_owner_total(self.h, int(n)), 'sbd_owner_total')

    def expand_counts(self, nchunk=1):
        """Wait for the expansion; (nchunk, world) records per exchange chunk and owner, raw total."""
        C = self.C
        counts = np.zeros(nchunk * self.world_x, np.int64)
        nraw = C.c_int64()
        self._chk(self.lib.sbd_expand_counts(self.h, int(nchunk), counts.ctypes.data, C.byref(nraw)),
                  'sbd_expand_counts')
        self.owner_counts = counts.reshape(nchunk, self.world_x).sum(axis=0)
        return counts.reshape(nchunk, self.world_x), nraw.value

    def expand_defer(self):
        """World 1: go on without waiting for the expansion (raw_total() after the next wait)."""
        self._chk(self.lib.sbd_expand_defer(self.h), 'sbd_expand_defer')

    def raw_total(self) -> int:
        nraw = self.C.c_int64()
        self._chk(self.lib.sbd_raw_total(self.h, self.C.byref(nraw)), 'sbd_raw_total')
        return nraw.value

    def _empty(self, n, dtype=torch.int64):
        return torch.empty(int(n), dtype=dtype, device=self.device)

    def pack(self):
        n = int(self.owner_counts.sum())
        key = self._empty(n)
        self._chk(self.lib.sbd_pack(self.h, key.data_ptr(), None), 'sbd_pack')
        return key

    def answer_buffer(self, n):
        return self._empty(max(int(n), 1), torch.uint8)[:int(n)]

    def owner_begin(self, n_total, src_base):
        sb = np.ascontiguousarray(np.asarray(src_base, dtype=np.int64))
        self._chk(self.lib.sbd_owner_begin(self.h, int(n_total), len(sb), sb.ctypes.data), 'sbd_owner_begin')

    def owner_claim(self, rkey, starts, bases, ret):
        st = np.ascontiguousarray(starts, dtype=np.int64)
        ba = np.ascontiguousarray(bases, dtype=np.int64)
        self._chk(self.lib.sbd_owner_claim(self.h, rkey.data_ptr() if rkey.numel() else None, rkey.numel(), len(st),
                                           st.ctypes.data, ba.ctypes.data, ret.data_ptr()), 'sbd_owner_claim')

    def owner_finish(self, ret):
        self._chk(self.lib.sbd_owner_finish(self.h, ret.data_ptr()), 'sbd_owner_finish')

    def record_buffer(self, n):
        """The turn's receive buffer of record keys (global-order claims: every part lands in it): one buffer kept
        across turns and grown only when a turn needs more, so the caching allocator is not asked for a new
        multi-GB block whenever the bound moves (reuse is ordered like the allocator's: the previous turn's claims
        finished on the stream before this turn's first part can arrive)."""
        n = max(int(n), 1)
        if getattr(self, '_rbuf', None) is None or self._rbuf.numel() < n:
            self._rbuf = torch.empty(n + n // 8, dtype=torch.int64, device=self.device)
        return self._rbuf[:n]

    def ret_buffer(self, n):
        """The turn's claim answers (one byte per received record), kept across turns like record_buffer."""
        n = max(int(n), 1)
        if getattr(self, '_abuf', None) is None or self._abuf.numel() < n:
            self._abuf = torch.empty(n + n // 8, dtype=torch.uint8, device=self.device)
        return self._abuf[:n]

    def owner_claim_all(self, rbuf, n_total, v_start, p_start, ret):
        vs = np.ascontiguousarray(v_start, dtype=np.int64)
        ps = np.ascontiguousarray(p_start, dtype=np.int64)
        self._chk(self.lib.sbd_owner_claim_all(self.h, rbuf.data_ptr() if n_total else None, int(n_total), len(vs),
                                               vs.ctypes.data, ps.ctypes.data, ret.data_ptr() if n_total else None),
                  'sbd_owner_claim_all')

    def owner_claim_part(self, j, rbuf, v_begin, v_end, v_start, p_start, ret):
        """Part j's records [v_begin, v_end) claimed in global order (on the claim stream: the caller's current one)."""
        vs = np.ascontiguousarray(v_start, dtype=np.int64)
        ps = np.ascontiguousarray(p_start, dtype=np.int64)
        n = int(v_end) > int(v_begin)
        self._chk(self.lib.sbd_owner_claim_part(self.h, int(j), rbuf.data_ptr() if n else None, int(v_begin), int(v_end),
                                                len(vs), vs.ctypes.data, ps.ctypes.data, ret.data_ptr() if n else None),
                  'sbd_owner_claim_part')

    def block_counts(self, bounds):
        """Survivors per local block (device int64, after apply)."""
        bd = np.ascontiguousarray(np.asarray(bounds, dtype=np.int64))
        out = torch.zeros(len(bd) - 1, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_block_counts(self.h, len(bd) - 1, bd.ctypes.data, out.data_ptr()), 'sbd_block_counts')
        return out

    def pack_bits(self, src, dst):
        """dst (ceil(n/8) bytes) <- the n answer bytes of src as bits (bit k of byte i = src[8i + k])."""
        if src.numel():
            self._chk(self.lib.sbd_pack_bits(self.h, src.data_ptr(), src.numel(), dst.data_ptr()), 'sbd_pack_bits')

    def unpack_bits(self, src, dst):
        if dst.numel():
            self._chk(self.lib.sbd_unpack_bits(self.h, src.data_ptr(), dst.numel(), dst.data_ptr()), 'sbd_unpack_bits')

    def _bits_segs(self, fn, src, segs, dst):
        segs = [x for x in segs if x[1] > 0]
        if not segs:
            return
        so, ln, do = (np.ascontiguousarray([x[i] for x in segs], dtype=np.int64) for i in range(3))
        self._chk(fn(self.h, src.data_ptr(), len(segs), so.ctypes.data, ln.ctypes.data, dst.data_ptr(), do.ctypes.data),
                  fn.__name__)

    def pack_bits_segs(self, src, segs, dst):
        """For every (src offset, n, dst offset) in segs: the n answer bytes at src + offset as bits at dst +
        offset (k_bits_segs: all segments in one launch)."""
        self._bits_segs(self.lib.sbd_pack_bits_segs, src, segs, dst)

    def unpack_bits_segs(self, src, segs, dst):
        """The inverse: (src bit-byte offset, n answer bytes, dst offset) per segment, one launch."""
        self._bits_segs(self.lib.sbd_unpack_bits_segs, src, segs, dst)

    def apply(self, back):
        """Survivor masks from the answers; this rank's unique count as a device int64 (no wait)."""
        n = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_apply(self.h, back.data_ptr(), n.data_ptr()), 'sbd_apply')
        return n

    def apply_finish(self, n_loc):
        self._chk(self.lib.sbd_apply_finish(self.h, int(n_loc)), 'sbd_apply_finish')

    def noise_info(self):
        out = np.zeros(8, np.uint64)
        self._chk(self.lib.sbd_noise_info(self.h, out.ctypes.data), 'sbd_noise_info')
        self.P, self.S = int(out[0]), int(out[5])
        return [int(x) for x in out]

    def noise_chunk(self, slot):
        counts = torch.empty(self.P * self.S, dtype=torch.int32, device=self.device)
        self._chk(self.lib.sbd_noise_chunk(self.h, int(slot), counts.data_ptr()), 'sbd_noise_chunk')
        return counts

    def noise_sync(self):
        self._chk(self.lib.sbd_noise_sync(self.h), 'sbd_noise_sync')

    def noise_pack(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        wins = torch.empty((len(idx), 624), dtype=torch.int32, device=self.device)
        if len(idx):
            self._chk(self.lib.sbd_noise_pack(self.h, len(idx), idx.ctypes.data, wins.data_ptr()), 'sbd_noise_pack')
        return wins

    def noise_fill(self, wins, acc0, a, e):
        acc0 = np.ascontiguousarray(acc0, dtype=np.uint64)
        if len(acc0):
            self._chk(self.lib.sbd_noise_fill(self.h, len(acc0), wins.data_ptr(), acc0.ctypes.data, int(a), int(e)),
                      'sbd_noise_fill')

    def noise_fill_ranges(self, wins, acc0, ranges):
        """ranges: (a, b, dst) — draws [a, b) kept at ring positions dst.. (block-cyclic slices)."""
        acc0 = np.ascontiguousarray(acc0, dtype=np.uint64)
        if not len(acc0) or not ranges:
            return
        a, b, d = (np.ascontiguousarray([x[i] for x in ranges], dtype=np.uint64) for i in range(3))
        self._chk(self.lib.sbd_noise_fill_ranges(self.h, len(acc0), wins.data_ptr(), acc0.ctypes.data, len(a),
                                                 a.ctypes.data, b.ctypes.data, d.ctypes.data), 'sbd_noise_fill_ranges')

    def emit(self, k_off, N, off):
        self._chk(self.lib.sbd_emit(self.h, int(k_off), int(N), int(off)), 'sbd_emit')

    def key_range(self):
        rng = torch.empty(2, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_key_range(self.h, rng.data_ptr()), 'sbd_key_range')
        return rng

    def sel_begin(self, pos, rng):
        if getattr(self, 'sel_h', None) is None or self.sel_h.numel() != len(pos) * 1024:
            self.sel_h = torch.zeros(len(pos) * 1024, dtype=torch.int64, device=self.device)
            self.sel_eqbuf = torch.zeros(1, dtype=torch.int64, device=self.device)
        p = np.ascontiguousarray(np.array(pos, dtype=np.int64))
        self._chk(self.lib.sbd_sel_begin(self.h, len(pos), p.ctypes.data, rng.data_ptr()), 'sbd_sel_begin')

    def sel_begin_approx(self, pos, rng, nexact, fmax):
        self.sel_begin(pos, rng)   # (the histogram buffers)
        p = np.ascontiguousarray(np.array(pos, dtype=np.int64))
        self._chk(self.lib.sbd_sel_begin_approx(self.h, len(pos), p.ctypes.data, rng.data_ptr(), int(nexact), int(fmax)),
                  'sbd_sel_begin_approx')

    def sel_hist(self, src):
        self._chk(self.lib.sbd_sel_hist(self.h, int(src), self.sel_h.data_ptr()), 'sbd_sel_hist')
        return self.sel_h

    def sel_pick(self, h):
        self._chk(self.lib.sbd_sel_pick(self.h, h.data_ptr()), 'sbd_sel_pick')

    def sel_compact(self):
        self._chk(self.lib.sbd_sel_compact(self.h), 'sbd_sel_compact')

    def sel_eq(self):
        self._chk(self.lib.sbd_sel_eq(self.h, self.sel_eqbuf.data_ptr()), 'sbd_sel_eq')
        return self.sel_eqbuf

    def sel_eq_blocks(self, qstart):
        """The keep boundary's ties per local block (device int64, nb)."""
        q = np.ascontiguousarray(np.asarray(qstart, dtype=np.int64))
        out = torch.zeros(len(q) - 1, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_sel_eq_blocks(self.h, len(q) - 1, q.ctypes.data, out.data_ptr()), 'sbd_sel_eq_blocks')
        return out

    def partition_blocks(self, has_top, eq_all, rank, G, nb, qstart=None):
        """Destinations (rank, block) of the kept records; per-digit counts (device int64, G * nb).  qstart (the blocks'
        local next_queue starts): the kept records per (local block, digit) are counted on the way (dest_subcounts)."""
        counts = torch.zeros(G * nb, dtype=torch.int64, device=self.device)
        q = np.ascontiguousarray(np.asarray(qstart, dtype=np.int64)) if qstart is not None else None
        self._sub = torch.empty(nb * G * nb, dtype=torch.int64, device=self.device) if q is not None else None
        self._chk(self.lib.sbd_partition_blocks(self.h, int(bool(has_top)), eq_all.data_ptr() if eq_all is not None else None,
                                                int(rank), int(G), int(nb), counts.data_ptr(),
                                                q.ctypes.data if q is not None else None,
                                                self._sub.data_ptr() if q is not None else None), 'sbd_partition_blocks')
        return counts

    def dest_subcounts(self, qstart, D):
        """Kept records per (local block, digit): device int64 (nb, D) — counted by partition_blocks when it had them."""
        if getattr(self, '_sub', None) is not None:
            sub, self._sub = self._sub, None
            return sub
        q = np.ascontiguousarray(np.asarray(qstart, dtype=np.int64))
        out = torch.zeros((len(q) - 1) * int(D), dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_dest_subcounts(self.h, len(q) - 1, q.ctypes.data, int(D), out.data_ptr()),
                  'sbd_dest_subcounts')
        return out

    def partition(self, has_top, eq_all, rank, nsplit, G):
        """Kept records' destinations; per-destination counts as a device int64 tensor (no wait)."""
        counts = torch.zeros(G, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_partition(self.h, int(bool(has_top)), eq_all.data_ptr() if eq_all is not None else None,
                                         int(rank), int(nsplit), int(G), counts.data_ptr()), 'sbd_partition')
        return counts

    def partition_bfs(self, k_off, N, G):
        counts = torch.zeros(G, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_partition_bfs(self.h, int(k_off), int(N), int(G), counts.data_ptr()),
                  'sbd_partition_bfs')
        return counts

    def pack_kept_grouped(self, n_rows, ndig=None):
        """Grouped kept records (sbd_pack_kept_grouped): (int32 buffer of 22 bytes per local survivor, device
        int64 (C_d, G_d) pairs per destination digit — ndig of them, default world), enqueued before the counts reach
        the host."""
        D = int(ndig or self.world)
        cap = 22 * int(n_rows) // 4 + 2 * D + 2
        buf = torch.empty(max(cap, 1), dtype=torch.int32, device=self.device)
        cnt2 = torch.zeros(2 * D, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_pack_kept_grouped(self.h, buf.data_ptr(), cap, cnt2.data_ptr()), 'sbd_pack_kept_grouped')
        return buf, cnt2

    def unpack_kept(self, rbuf, bases, groups, children, perm=None, pmap=None):
        """The received groups (segments at u32 offsets bases, in order) as (n, 5) int32 records; perm: (source child,
        destination record) run starts, pmap: (sender parent number, global rank) run starts (block-cyclic slices)."""
        n = int(np.sum(children))
        rec = torch.empty((max(n, 1), 5), dtype=torch.int32, device=self.device)
        b = np.ascontiguousarray(bases, dtype=np.int64)
        g = np.ascontiguousarray(groups, dtype=np.int64)
        c = np.ascontiguousarray(children, dtype=np.int64)
        pm = np.ascontiguousarray(np.asarray(perm, dtype=np.int64).reshape(-1)) if perm else np.zeros(2, np.int64)
        mp = np.ascontiguousarray(np.asarray(pmap, dtype=np.int64).reshape(-1)) if pmap else np.zeros(2, np.int64)
        P = self.C.POINTER(self.C.c_int64)
        self._chk(self.lib.sbd_unpack_kept(self.h, rbuf.data_ptr() if rbuf.numel() else None, len(b),
                                           b.ctypes.data_as(P), g.ctypes.data_as(P), c.ctypes.data_as(P),
                                           rec.data_ptr(), len(perm) if perm else 0, pm.ctypes.data,
                                           len(pmap) if pmap else 0, mp.ctypes.data), 'sbd_unpack_kept')
        return rec[:n]

    def pack_kept(self, n_rows, rec20=False):
        """Kept records grouped by destination into a buffer of n_rows (>= the kept count: the local
        next_queue size), enqueued before the counts reach the host."""
        # 3 words (lo, hi, parent | draw << 32; with owner emission parent | draw << 25 | position << 32), or with
        # rec20 five u32 (lo, hi, parent | draw << 25): the receiver re-scores them
        rec20 = bool(rec20) and not self.oe
        if rec20:
            rec = torch.empty((max(int(n_rows), 1), 5), dtype=torch.int32, device=self.device)
        else:
            rec = torch.empty((max(int(n_rows), 1), 3), dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_pack_kept(self.h, rec.data_ptr() if n_rows else None, int(rec20)), 'sbd_pack_kept')
        return rec

    # ---------------------------------------------------------------- card-set ownership (sb_mig.inc)
    def keypass_ms(self) -> float:
        out = np.zeros(1, np.float32)
        self._chk(self.lib.sbd_keypass_ms(self.h, out.ctypes.data), 'sbd_keypass_ms')
        return float(out[0])

    def mig_launch(self):
        self._chk(self.lib.sbd_mig_launch(self.h, int(self.world)), 'sbd_mig_launch')

    def mig_counts(self) -> np.ndarray:
        """The slice's parents per card-set owner, then their raw children per owner (2 x world)."""
        out = np.zeros(2 * self.world, np.int64)
        self._chk(self.lib.sbd_mig_counts(self.h, out.ctypes.data), 'sbd_mig_counts')
        return out

    def mig_pack(self, goff, n):
        rows = torch.empty((max(int(n), 1), 5), dtype=torch.int32, device=self.device)
        self._chk(self.lib.sbd_mig_pack(self.h, int(goff), rows.data_ptr() if n else None), 'sbd_mig_pack')
        return rows[:int(n)]

    def mig_expand(self, rflat, n_exp, n_global):
        self.world_x = self.world
        self._chk(self.lib.sbd_mig_expand(self.h, int(self.world), int(self.parts), int(n_global),
                                          rflat.data_ptr() if n_exp else None, int(n_exp)), 'sbd_mig_expand')
        self.n_exp = int(n_exp)

    def mig_claim(self, rrec, ans_base, ret):
        m = rrec.numel() // 3
        self._chk(self.lib.sbd_mig_claim(self.h, rrec.data_ptr() if m else None, int(m), int(ans_base),
                                         ret.data_ptr() if m else None), 'sbd_mig_claim')

    def bits_buffer(self, nbytes):
        """A zeroed byte stream of nbytes plus two words of slack (the kernels touch the word after a segment's
        last bit); the caller slices [0, nbytes)."""
        return torch.zeros(((int(nbytes) + 7) // 8 + 2) * 8, dtype=torch.uint8, device=self.device)

    def mig_apply(self, back, bits, seg_start, seg_byte, keep=False):   # keep: implied by the engine's flags bit 9
        st = np.ascontiguousarray(seg_start, dtype=np.int64)
        sb = np.ascontiguousarray(seg_byte, dtype=np.int64)
        self._chk(self.lib.sbd_mig_apply(self.h, back.data_ptr() if back.numel() else None, bits.data_ptr(),
                                         len(sb), st.ctypes.data, sb.ctypes.data), 'sbd_mig_apply')

    def mig_place(self, rbits, group_start, byte_base):
        n = torch.zeros(1, dtype=torch.int64, device=self.device)
        gs = np.ascontiguousarray(group_start, dtype=np.int64)
        bb = np.ascontiguousarray(byte_base, dtype=np.int64)
        self._chk(self.lib.sbd_mig_place(self.h, rbits.data_ptr(), len(bb), gs.ctypes.data, bb.ctypes.data,
                                         n.data_ptr()), 'sbd_mig_place')
        return n

    # ---------------------------------------------------------------- owner emission (sb_oe.inc)
    def oe_pack(self, k_off, N, so, n_unique_local):
        """Range side: rows' global offsets (u32) and their survivors' noise draws (bytes), rows' order; the noise
        bytes per owner on the host (waits for them)."""
        n = self.n_local()
        rgoff = self._empty(max(n, 1), torch.int32)[:n]
        heur = getattr(self, 'heur', True)
        rnoise = self._empty(max(int(n_unique_local), 1), torch.uint8)[:int(n_unique_local)]
        gs = np.ascontiguousarray(so, dtype=np.int64)
        nb = np.zeros(len(gs) - 1, np.int64)
        self._chk(self.lib.sbd_oe_pack(self.h, int(k_off), int(N), rgoff.data_ptr() if n else None,
                                       rnoise.data_ptr() if heur else None, len(gs) - 1, gs.ctypes.data, nb.ctypes.data),
                  'sbd_oe_pack')
        return rgoff, rnoise, nb

    def oe_counts(self, ro):
        """Expand side: survivors per source segment (host; waits), their offsets on the device."""
        gs = np.ascontiguousarray(ro, dtype=np.int64)
        out = np.zeros(len(gs) - 1, np.int64)
        self._chk(self.lib.sbd_oe_counts(self.h, len(gs) - 1, gs.ctypes.data, out.ctypes.data), 'sbd_oe_counts')
        self._oe_n = int(out.sum())
        return out

    def u32_buffer(self, n):
        return self._empty(max(int(n), 1), torch.int32)[:int(n)]

    def byte_buffer(self, n):
        return self._empty(max(int(n), 1), torch.uint8)[:int(n)]

    def oe_emit(self, xgoff, xnoise):
        self._chk(self.lib.sbd_oe_emit(self.h, xgoff.data_ptr() if xgoff.numel() else None,
                                       xnoise.data_ptr() if xnoise is not None and xnoise.numel() else None),
                  'sbd_oe_emit')

    def oe_n(self):
        return self._oe_n

    def oe_ties(self):
        C = self.C
        cnt, need = C.c_int64(), C.c_int64()
        self._chk(self.lib.sbd_oe_ties(self.h, C.byref(cnt), C.byref(need)), 'sbd_oe_ties')
        pos = np.zeros(cnt.value, np.int64)
        if cnt.value:
            self._chk(self.lib.sbd_oe_tie_read(self.h, pos.ctypes.data, cnt.value), 'sbd_oe_tie_read')
        return pos, need.value

    def oe_partition(self, has_top, pstar, nsplit, G):
        counts = torch.zeros(G, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_oe_partition(self.h, int(bool(has_top)), int(pstar), int(nsplit), int(G), counts.data_ptr()),
                  'sbd_oe_partition')
        return counts

    def oe_partition_bfs(self, N, G):
        counts = torch.zeros(G, dtype=torch.int64, device=self.device)
        self._chk(self.lib.sbd_oe_partition_bfs(self.h, int(N), int(G), counts.data_ptr()), 'sbd_oe_partition_bfs')
        return counts

    def oe_segments(self, seg_start):
        gs = np.ascontiguousarray(seg_start, dtype=np.int64)
        self._chk(self.lib.sbd_oe_segments(self.h, len(gs) - 1, gs.ctypes.data), 'sbd_oe_segments')

    def receive(self, rec, heur):
        self._chk(self.lib.sbd_receive(self.h, rec.data_ptr() if rec.numel() else None, rec.shape[0], int(bool(heur))),
                  'sbd_receive')

"""RCCL's completion contract for splendor_amd.dist.Comm, on the GPU (TEST INFRASTRUCTURE).

The 8-GPU job runs Comm's RCCL branches (``cpu_coll`` False: device tensors, ``all_to_all(..., async_op=True)`` whose
receive buffer is valid only after ``wait(handle)``, in-place ``all_reduce``, list ``all_to_all`` into views) against
the HIP engine's two streams (the engine stream and the claim stream, dist.py ``_exchange_parts``).  RCCL refuses
two ranks on one device, so on a one-GPU box those branches cannot run with a world of more than one.  This double
runs them with the device-side semantics RCCL has, the data itself moving over gloo:

* a collective reads its inputs in the order of the stream current at the call (the inputs are copied to the host
  on that stream: every kernel enqueued on it before the call has run, nothing else is waited for);
* its outputs land on a side stream, behind a delay kernel (``torch.cuda._sleep``), over a poison pattern written
  first: a consumer that reads a receive buffer without being ordered after the collective reads poison, not data;
* a synchronous collective orders the current stream after the landing (``wait_event``), as RCCL's stream
  semantics do; an asynchronous ``alltoall_pieces`` does so only in ``wait(handle)``, on the stream current at the
  wait — a wait on the wrong stream leaves the consumer unordered;
* the send pieces of an asynchronous all_to_all must not change before it completes: the side stream compares them
  with their contents at the call once the delay has run, and ``check_step`` fails on any difference;
* every handle is waited for within its step (``check_step``).
"""
import torch
import torch.distributed as dist

from splendor_amd.dist import Comm

_POISON = {torch.uint8: 0xA5, torch.int32: -0x5A5A5A5B, torch.int64: -0x5A5A5A5A5A5A5A5B}


class _Handle:
    def __init__(self, out, done):
        self.out, self.done = out, done
        self.waited = False


class DeviceDeferredComm(Comm):
    def __init__(self, device, delay_cycles=200_000):
        super().__init__(device)
        self.cpu_coll = False                 # Comm's RCCL branches
        self.side = torch.cuda.Stream(device)
        self.delay = int(delay_cycles)
        self.bad = torch.zeros(1, dtype=torch.int64, device=device)   # send pieces changed before completion
        self.outstanding = []
        self.deferred_calls = 0
        self.waits = 0
        self.landings = 0

    # ------------------------------------------------------------------ the device-side contract
    @staticmethod
    def _host(t):
        """t as the collective reads it: on the current stream (the host waits for that stream only)."""
        return t.detach().to('cpu')

    def _land(self, pairs, guard=()):
        """dst <- host data for every (dst, host) pair on the side stream, after the current stream's work so far:
        poison, delay, data.  guard: (piece, its contents at the call) pairs compared after the delay.  Returns the
        landing's completion event."""
        cur = torch.cuda.current_stream(self.device)
        start = torch.cuda.Event()
        start.record(cur)
        self.side.wait_event(start)
        with torch.cuda.stream(self.side):
            staged = [(d, h.to(self.device)) for d, h in pairs if d.numel()]
            for d, _ in staged:
                d.fill_(_POISON[d.dtype])
            torch.cuda._sleep(self.delay)
            for p, s in guard:
                if p.numel():
                    self.bad += (p.reshape(-1) != s.reshape(-1)).sum()
            for d, x in staged:
                d.copy_(x.reshape(d.shape))
                d.record_stream(self.side)
                x.record_stream(self.side)
            for p, s in guard:
                p.record_stream(self.side)
                s.record_stream(self.side)
        done = torch.cuda.Event()
        done.record(self.side)
        self.landings += 1
        return done

    def _order(self, done):
        torch.cuda.current_stream(self.device).wait_event(done)

    def check_step(self):
        """Call between steps: every handle waited for, no send piece changed in flight."""
        assert not self.outstanding, f'{len(self.outstanding)} all_to_all handle(s) left unwaited'
        torch.cuda.synchronize(self.device)
        assert int(self.bad.item()) == 0, 'a send piece changed before its all_to_all completed'

    # ------------------------------------------------------------------ Comm's device collectives
    def _gather_flat(self, t):
        s = self._host(t).reshape(-1)
        if self.world == 1:
            return t.reshape(-1)
        h = torch.empty(self.world * s.numel(), dtype=s.dtype)
        dist.all_gather_into_tensor(h, s)
        out = torch.empty(h.numel(), dtype=t.dtype, device=self.device)
        self._order(self._land([(out, h)]))
        return out

    def alltoall_counts_dev(self, counts):
        send = self._host(counts)
        if self.world == 1:
            c = send.numpy()
            return c, c
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send)
        return send.numpy(), recv.numpy()

    def alltoall_counts(self, counts):
        send = torch.as_tensor(counts, dtype=torch.int64).contiguous()
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send)
        return recv.numpy()

    def alltoall(self, send, send_counts, recv_counts, what='other'):
        row = send.element_size() * (int(send[0].numel()) if send.dim() > 1 and send.shape[0] else 1)
        self.acct(what, row * (int(sum(send_counts)) - int(send_counts[self.rank])))
        s = self._host(send)
        r = torch.empty((int(sum(recv_counts)),) + tuple(send.shape[1:]), dtype=send.dtype)
        dist.all_to_all_single(r, s, [int(x) for x in recv_counts], [int(x) for x in send_counts])
        out = torch.empty(r.shape, dtype=send.dtype, device=self.device)
        self._order(self._land([(out, r)]))
        return out

    def alltoall_pieces(self, pieces, recv_sizes, what='other', out=None):
        self.acct(what, self._remote(pieces))
        snap = [self._host(p) for p in pieces]
        send = torch.cat([x.reshape(-1) for x in snap])
        r = torch.empty(int(sum(recv_sizes)), dtype=pieces[0].dtype)
        dist.all_to_all_single(r, send, [int(x) for x in recv_sizes], [int(p.numel()) for p in pieces])
        if out is None:
            out = torch.empty(int(sum(recv_sizes)), dtype=pieces[0].dtype, device=self.device)
        guard = [(p, x.to(self.device)) for p, x in zip(pieces, snap)]
        h = _Handle(out, self._land([(out, r)], guard))
        self.outstanding.append(h)
        self.deferred_calls += 1
        return out, h

    def wait(self, handle):
        if handle is None:
            return
        assert not handle.waited, 'handle waited for twice'
        self._order(handle.done)   # the stream current at the wait, as RCCL's work.wait()
        handle.waited = True
        self.outstanding.remove(handle)
        self.waits += 1

    def alltoall_into(self, pieces, outs, what='other'):
        self.acct(what, self._remote(pieces))
        send = torch.cat([self._host(p).reshape(-1) for p in pieces])
        rows = [int(o.numel()) for o in outs]
        r = torch.empty(sum(rows), dtype=send.dtype)
        dist.all_to_all_single(r, send, rows, [int(p.numel()) for p in pieces])
        self._order(self._land(list(zip(outs, r.split(rows)))))

    def allreduce_tensor(self, t, op=dist.ReduceOp.SUM, what='select all_reduce'):
        if self.world == 1:
            return
        self.acct(what, 2 * (self.world - 1) * t.numel() * t.element_size() // self.world)
        x = self._host(t)
        dist.all_reduce(x, op=op)
        self._order(self._land([(t, x)]))

    def allreduce(self, arr, op):
        t = torch.as_tensor(arr, dtype=torch.int64).contiguous().clone()
        dist.all_reduce(t, op=op)
        return t.numpy()

    def allgather_int(self, v):
        import numpy as np
        if self.world == 1:
            return np.array([int(v)], dtype=np.int64)
        t = torch.tensor([int(v)], dtype=torch.int64)
        out = torch.empty(self.world, dtype=torch.int64)
        dist.all_gather_into_tensor(out, t)
        return out.numpy()

    def broadcast_ints(self, vals, src):
        t = torch.tensor([int(v) for v in vals], dtype=torch.int64)
        dist.broadcast(t, src)
        return [int(x) for x in t.tolist()]

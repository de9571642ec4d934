"""RCCL completion semantics for splendor_amd.dist.Comm on CPU (TEST INFRASTRUCTURE).

Comm has two sets of branches: gloo (``cpu_coll``: every collective staged through the host and complete
on return) and RCCL (``nccl``: device tensors, ``all_to_all(..., async_op=True)`` whose receive buffer is
valid only after ``wait(handle)``, in-place ``all_reduce``, list ``all_to_all`` into views).  The round-end
8-GPU run is the first place the RCCL branches would run for real; this double runs them on CPU over gloo
with RCCL's contract enforced, so an ordering bug in the protocol shows up as a wrong beam here:

* ``cpu_coll`` is False, so every call takes the non-gloo branch of Comm;
* ``alltoall_pieces`` returns a deferred handle: the receive buffer holds a poison pattern until
  ``wait(handle)`` (a consumer that reads before waiting claims poisoned keys), and the send pieces must
  not change between the call and the wait (RCCL reads them asynchronously: checked at ``wait``);
* every handle must be waited for before the step ends (``outstanding``; the test checks it per step);
* list all_to_all (``alltoall_into``), which gloo lacks, is emulated with all_to_all_single: a synchronous
  RCCL collective is ordered before later work on the stream, which on CPU is plain completion.
"""
import torch
import torch.distributed as dist

from splendor_amd.dist import Comm

_POISON = {torch.uint8: 0xA5, torch.int32: -0x5A5A5A5B, torch.int64: -0x5A5A5A5A5A5A5A5B}


class _Deferred:
    def __init__(self, out, data, pieces, snap):
        self.out, self.data, self.pieces, self.snap = out, data, pieces, snap
        self.done = False


class DeferredComm(Comm):
    def __init__(self, device):
        super().__init__(device)
        self.cpu_coll = False
        self.outstanding = []
        self.deferred_calls = 0
        self.waits = 0

    def alltoall_pieces(self, pieces, recv_sizes, what='other', out=None):
        self.acct(what, self._remote(pieces))
        snap = [p.clone() for p in pieces]
        send = torch.cat([p.reshape(-1) for p in snap]) if snap else torch.zeros(0)
        data = torch.empty(int(sum(recv_sizes)), dtype=pieces[0].dtype)
        dist.all_to_all_single(data, send, [int(x) for x in recv_sizes], [int(p.numel()) for p in pieces])
        if out is None:
            out = torch.empty(int(sum(recv_sizes)), dtype=pieces[0].dtype)
        out.fill_(_POISON[pieces[0].dtype])
        h = _Deferred(out, data, list(pieces), snap)
        self.outstanding.append(h)
        self.deferred_calls += 1
        return out, h

    def wait(self, handle):
        if handle is None:
            return
        assert not handle.done, 'handle waited for twice'
        for p, s in zip(handle.pieces, handle.snap):
            assert torch.equal(p, s), 'a send piece changed before its all_to_all completed'
        handle.out.copy_(handle.data)
        handle.done = True
        self.outstanding.remove(handle)
        self.waits += 1

    def alltoall_into(self, pieces, outs, what='other'):
        self.acct(what, self._remote(pieces))
        send = torch.cat([p.reshape(-1) for p in pieces])
        rows = [int(o.numel()) for o in outs]
        r = torch.empty(sum(rows), dtype=send.dtype)
        dist.all_to_all_single(r, send, rows, [int(p.numel()) for p in pieces])
        for o, x in zip(outs, r.split(rows)):
            o.copy_(x.reshape(o.shape))

"""A one-process stand-in for an N-rank RCCL group, for the pipelined
assembly (core/sharding.PipelinedAssembly) on a one-GPU box.

RCCL's ``all_gather_into_tensor(out, inp, async_op=True)`` on ROCm: the
collective's own stream waits on the issuing stream, the gather runs there,
and the returned work's ``wait()`` makes the then-current stream wait on it.
``EmuComm.all_gather_into`` does the same with a real second stream:

* its stream waits on the caller's current stream (an event);
* a spin kernel (``torch.cuda._sleep``) stands in for the link time of the
  bytes this rank would receive (``recv_bytes / rate``), optionally
  followed by a device copy of those bytes (the HBM writes a gather makes);
* ``expected`` (test mode): the other ranks' pieces of the round are
  written from it, and the rank's own piece is snapshotted into ``sent``
  at the point the collective would have read it — so a collective that
  ran before its piece was computed, or a caller that read the result
  before the gather finished, shows up as a mismatch.

Returns a work object whose ``wait()`` has ProcessGroupNCCL's semantics.
Test and measurement infrastructure only; the product path uses
``core/sharding.Comm``.
"""
import torch


class _Work:
    def __init__(self, ev, device):
        self.ev = ev
        self.device = device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.ev)


def sleep_cycles_per_us(device):
    """Calibrate torch.cuda._sleep (cycles) against wall time."""
    with torch.cuda.device(device):
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        cyc = 2_000_000
        best = None
        for _ in range(3):
            a.record()
            torch.cuda._sleep(cyc)
            b.record()
            b.synchronize()
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
        return cyc / (best * 1e3)


class EmuComm:
    def __init__(self, world, rank, device, expected=None, base=None,
                 rate_gbps=None, copy=False, delay_us=0.0, cyc_per_us=None):
        self.group = None
        self.world = world
        self.rank = rank
        self.backend = 'emulated'
        self.host_staged = False
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.expected = expected
        self.base = base          # the padded output tensor (test mode)
        self.rate = rate_gbps
        self.copy = copy
        self.delay_us = delay_us
        self.cyc = cyc_per_us or (sleep_cycles_per_us(self.device)
                                  if (rate_gbps or delay_us) else 0.0)
        self.sent = []            # (offset, snapshot of own piece)
        self.calls = 0
        self._scratch = None

    def all_gather_into(self, out, inp, async_op=False):
        self.calls += 1
        cur = torch.cuda.current_stream(self.device)
        st = self.stream
        st.wait_stream(cur)
        L = out.numel()
        pc = inp.numel()
        recv = (self.world - 1) * pc * out.element_size()
        with torch.cuda.stream(st):
            us = self.delay_us + (recv / (self.rate * 1e3) if self.rate
                                  else 0.0)
            if us > 0:
                torch.cuda._sleep(int(us * self.cyc))
            if self.copy and recv:
                if self._scratch is None or self._scratch.numel() < \
                        (self.world - 1) * pc:
                    self._scratch = torch.empty((self.world - 1) * pc,
                                                dtype=out.dtype,
                                                device=self.device)
                # the received bytes land in HBM (other ranks' slots)
                k = 0
                for r in range(self.world):
                    if r != self.rank:
                        out[r * pc:(r + 1) * pc].copy_(
                            self._scratch[k * pc:(k + 1) * pc])
                        k += 1
            if self.expected is not None:
                off = (out.data_ptr() - self.base.data_ptr()) // \
                    out.element_size()
                own = off + self.rank * pc
                self.sent.append((own, inp.clone()))
                for r in range(self.world):
                    if r != self.rank:
                        a = off + r * pc
                        out[r * pc:(r + 1) * pc].copy_(
                            self.expected[a:a + pc])
            ev = torch.cuda.Event()
            ev.record(st)
        assert L == self.world * pc
        if not async_op:
            cur.wait_event(ev)
            return None
        return _Work(ev, self.device)

    def all_reduce_sum(self, t):
        return t

"""The stream-ordered flags of the data-parallel step (sae_flag_bump / sae_stream_wait_flag).

train.py's flag-gated all-reduce relies on two things that a one-rank RCCL run cannot
show, because a one-rank all-reduce reads nothing: (1) the communication stream really WAITS for the
flag (a wait that passed at once would let the all-reduce read a bucket before the backward wrote
it), and (2) the data the compute stream wrote before the flag bump -- from every CU, i.e. through
all eight XCDs' L2s -- is what a kernel on the waiting stream reads.  Here a producer stream sleeps
(sae_occupy_cus), fills a 256 MB buffer from every CU, bumps a flag; a consumer stream waits for the
flag and copies the buffer; every element of the copy must be the fill value, round after round."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_stream_wait_flag_orders_and_publishes(dev):
    import sae_vision_amd.ops as ops
    n = 64 * 1024 * 1024
    x = torch.zeros(n, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    prod, cons = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    for k in range(1, 6):
        with torch.cuda.stream(prod):
            ops.occupy_cus(prod, 256, 2000.0, lds_bytes=0)   # 2 ms: the consumer must not run ahead
            x.fill_(float(k))
            ops.flag_bump(flags, 1)
        ops.stream_wait_flag(cons, flags, 1, k)
        with torch.cuda.stream(cons):
            y.copy_(x)
            done = torch.cuda.Event()
            done.record(cons)
        done.synchronize()
        assert bool((y == float(k)).all()), f"round {k}: the consumer read {y.unique()[:4].tolist()}"
    torch.cuda.synchronize()
    assert flags.tolist() == [0, 5]


def test_flag_bump_captured_in_graph(dev):
    """A bump captured in a HIP graph runs once per replay (the step's epoch count)."""
    import sae_vision_amd.ops as ops
    flags = torch.zeros(3, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            ops.flag_bump(flags, 0)
            ops.flag_bump(flags, 2)
    for _ in range(4):
        g.replay()
    torch.cuda.synchronize()
    assert flags.tolist() == [4, 0, 4]

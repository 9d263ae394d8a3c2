"""Child process of tests/test_gpu_train_graph.py::test_world1_rccl_overlapped_step (GPU).

    python tests/world1_rccl_case.py <deit_ti_patch16 | cait>

The multi-rank step's collective path on one GPU: a one-rank RCCL group (backend nccl), the
bucket all-reduces on the communication stream, overlapped with the backward: gated by device flags
the captured (linear) backward graph bumps (train.py "flagged", the default), or with SAE_FLAGGED=0
forked inside ONE HIP graph with the rest of the step (train.py "overlap").  A one-rank SUM is the identity,
so losses and parameters must equal the no-collective graph step's bit for bit; the buckets must
all have been launched, the first before the backward finished.  Prints WORLD1_OK on success.
"""
import copy
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(model):
    import torch
    import torch.distributed as dist
    from sae_vision_amd import cait, ops, train, vit
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    if model == "cait":
        m_a = cait.create_cait("cait_xxs_24", 1000, torch.bfloat16, stoch_depth=False, device=dev)
    else:
        m_a = vit.create_model(model, 1000, torch.bfloat16, device=dev)
    m_b = copy.deepcopy(m_a)
    s_a = train.TrainStep(m_a, global_batch=8, device=dev, graph=True)
    assert s_a.collective == "none"
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)   # as train.init_distributed
    s_b = None
    try:
        s_b = train.TrainStep(m_b, global_batch=8, device=dev, graph=True, bucket_cap_mb=4.0)
        assert s_b.collective == "overlap" and len(s_b._buckets) > 1
        order = []
        orig = s_b._launch_bucket
        s_b._launch_bucket = lambda bi: (order.append((bi, len(s_b._ready))), orig(bi))[1]
        g = torch.Generator(device=dev).manual_seed(3)
        data = [(torch.randn(8, 224, 224, 3, device=dev, generator=g),
                 torch.randint(0, 1000, (8,), device=dev, generator=g)) for _ in range(3)]
        la = [float(s_a(x, y)) for x, y in data]
        lb = [float(s_b(x, y)) for x, y in data]
        nb = len(s_b._buckets)
        assert sorted(bi for bi, _ in order[-nb:]) == list(range(nb))     # the captured backward's launches
        assert order[-nb][1] < len(s_b._params)                            # the first before the last gradient
        if os.environ.get("SAE_FLAGGED", "1") != "0":
            # flagged: a linear forward + backward graph with one flag bump per bucket, the optimizer's
            # graph, and the all-reduces issued per replay behind the flags (one per bucket per replay)
            assert s_b._flagged and s_b._g is not None and s_b._g_opt is not None and s_b.graph
            assert sorted(s_b._flag_order) == list(range(nb))
            torch.cuda.synchronize()
            assert s_b._flags.tolist() == [len(data)] * nb, s_b._flags.tolist()
        else:
            assert s_b._g is not None and s_b._g_opt is None and s_b.graph   # one graph, collectives inside
        assert la == lb, (la, lb)
        for (n, pa), pb in zip(m_a.named_parameters(), m_b.parameters()):
            assert torch.equal(pa, pb), n
    finally:
        # the captured graph holds RCCL collectives: it goes before the communicator
        if s_b is not None:
            s_b.close()
        s_a.close()
        dist.destroy_process_group()
        ops.set_sink_listener(None)
    print("WORLD1_OK", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])

"""Shared helpers of the GPU parity tests: run a batch through an NF's
C-ABI (vp_process_device via vigor_amd) and compare with the oracle."""
import numpy as np
import torch


def run_gpu(nf, frames, lens, in_dev, now, slot, affine=None):
    d = torch.device("cuda:0")
    f = torch.from_numpy(frames.copy()).to(d)
    l_ = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(d)
    if isinstance(in_dev, int):  # one port for the batch (vp_dev_batch.in_port)
        i_ = in_dev
    else:
        i_ = torch.from_numpy(in_dev.astype(np.uint16).view(np.int16)).to(d)
    o = torch.zeros(lens.shape[0], dtype=torch.int16, device=d)
    if affine is None:
        nt = torch.from_numpy(now.astype(np.int64)).to(d)
        nf.process_device(f, l_, i_, o, slot, now=nt)
    else:
        nf.process_device(f, l_, i_, o, slot, now0=affine[0],
                          now_step=affine[1])
    torch.cuda.synchronize()
    return f.cpu().numpy(), o.cpu().numpy().view(np.uint16)


def check_batches(nf, oracle, frames, lens, in_dev, now, slot, cuts,
                  affine=False, one_port=False):
    """Feed the trace as consecutive batches split at `cuts`; compare every
    batch's outputs with the oracle run over the same packets. one_port: each
    batch's packets share a port, passed as vp_dev_batch.in_port."""
    exp = frames.copy()
    exp_out = oracle.run(exp, lens, in_dev, now, slot)
    bounds = [0] + sorted(set(cuts)) + [lens.shape[0]]
    for a, b in zip(bounds[:-1], bounds[1:]):
        if a == b:
            continue
        fr = frames[a * slot:b * slot]
        aff = (int(now[a]), int(now[a + 1] - now[a]) if b - a > 1 else 1) \
            if affine else None
        ports = in_dev[a:b]
        if one_port:
            assert (ports == ports[0]).all()
            ports = int(ports[0])
        got, out = run_gpu(nf, fr, lens[a:b], ports, now[a:b], slot, aff)
        bad = np.nonzero(out != exp_out[a:b])[0]
        assert bad.size == 0, "out port mismatch at packets %s: %s vs %s" % (
            bad[:10] + a, out[bad[:10]], exp_out[a + bad[:10]])
        gf = got.reshape(b - a, slot)
        ef = exp[a * slot:b * slot].reshape(b - a, slot)
        badf = np.nonzero((gf != ef).any(axis=1))[0]
        assert badf.size == 0, "frame mismatch at packets %s" % (badf[:10] + a)

"""North-star end-to-end parity (BASELINE.json: "Mel/PCEN features and model
logits match the reference on identical clips within a stated fp32
tolerance").

Raw synthetic 3 s @ 48 kHz clips go through the product chain on the GPU,
    FrontEnd: normalize -> mix_up (fixed lambda) -> normalize -> STFT -> |X|^2
              -> mel -> PCEN + normalize_minmax          (acfe.train.FrontEnd)
    -> wr_resnet / wr_resnet_bird at the T1/I input 128 x 513 -> Keras CCE
    -> backward into the flat parameter arena (model + PCEN parameters),
and through the oracle chain on the CPU,
    of.normalize -> of.mix_up -> of.normalize -> of.raw_to_mel (float64 STFT)
    -> torch_ref.pcen_torch -> om.wr_resnet* (3 identical input channels)
    -> om.keras_loss -> autograd,
citing tfdataset.py:1916-1934 / :930-955 / :2007-2059, tfpcen.py:33-110,
resnet/wr_resnet.py:5-90, resnet/wr_resnet_bird.py:7-179,
audiomodel.py:1206-1223.

The wr_resnet case is config I's composed fp32 path (front end + PCEN +
wr_resnet forward at 128 x 513), here with its backward as well.

Tolerances (fp32 compute, eval-mode BN, dropout 0; oracle in float64):
  PCEN features   max |dev - ref| <= 2e-5 on the [-1, 1] output
  logits          rel-L2 <= 2e-5
  loss            |dev - ref| <= 2e-5 * max(1, |ref|)
  gradient arena  rel-L2 <= 2e-4 (model + PCEN parameters together)
  PCEN gradients  rel-L2 <= 1e-3 (four scalars summed over 3 x 128 x 513
                  elements through the batch-global min/max)
Measured on MI355X (r03a): features 1.2e-6; logits 2.3e-6 (wr_resnet) /
3.1e-7 (wr_resnet_bird); arena 1.1e-5 / 3.0e-5; PCEN gradients 1.7e-6 / 6.1e-5.
"""
import numpy as np
import pytest
import torch

from conftest import synth_clips

pytestmark = pytest.mark.gpu

B = 3
LAM = np.array([0.3, 0.0, 0.8])


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _oracle(kind, x1, x2, lam, weights, state_dict, pcen_params, tgt):
    """float64 oracle chain; returns (features [B,M,T], logits, loss, grads by name, pcen grad)."""
    from oracle import frontend as of
    from oracle import models as om
    from oracle.torch_ref import pcen_torch

    zeros = np.zeros((x1.shape[0], 1))
    mixed, _ = of.mix_up(of.normalize(x1), zeros, of.normalize(x2), zeros, lam)
    mel = of.raw_to_mel(of.normalize(mixed), weights)                     # [B, M, T] float64
    mel_btm = torch.from_numpy(np.ascontiguousarray(mel.transpose(0, 2, 1)))
    pp = pcen_params.detach().double().cpu().clone().requires_grad_(True)
    feats = pcen_torch(mel_btm, pp)                                        # [B, M, T]
    p = {k: v.detach().double().cpu().clone() for k, v in state_dict.items()}
    prm = {k: v.requires_grad_(True) for k, v in p.items() if "moving" not in k}
    st = {k: v for k, v in p.items() if "moving" in k}
    fwd = om.wr_resnet_bird if kind == "bird" else om.wr_resnet
    z = fwd(feats[:, None].repeat(1, 3, 1, 1), prm, False, st)
    loss = om.keras_loss(z, tgt, "cce")
    loss.backward()
    return feats.detach(), z.detach(), loss.detach(), {k: v.grad for k, v in prm.items()}, pp.grad


@pytest.mark.parametrize("kind", ["wrn", "bird"])
def test_raw_clips_to_logits_and_gradients(cuda, kind):
    from test_model_gpu import _build

    from acfe import ops
    from acfe.layers import ParamArena
    from acfe.train import FrontEnd, mix_labels

    classes = 2 if kind == "wrn" else 50
    x1 = synth_clips(B, seed=31)
    x2 = synth_clips(B, seed=41, noise_only_every=2)
    y1 = torch.zeros(B, classes)
    y2 = torch.zeros(B, classes)
    y1[torch.arange(B), torch.tensor([0, 1, 0]) % classes] = 1
    y2[torch.arange(B), torch.tensor([1, 1, 0]) % classes] = 1
    lam_t = torch.tensor(LAM, dtype=torch.float32)
    tgt = mix_labels(y1, y2, lam_t)

    # device chain
    m = _build(kind, (128, 513, 3), classes, torch.float32, cuda)
    fe = FrontEnd(n_mels=128, dtype=torch.float32, device=cuda, pcen=True).to(cuda)
    holder = torch.nn.ModuleList([fe, m])
    arena = ParamArena(holder, cuda)
    holder.eval()
    arena.zero_grad()
    feats = fe(torch.from_numpy(x1).to(cuda), torch.from_numpy(x2).to(cuda), lam_t.to(cuda))
    z = m(feats)
    loss, dz = ops.loss_and_grad(z, tgt.to(cuda), "cce")
    z.backward(dz)
    torch.cuda.synchronize()

    f_ref, z_ref, l_ref, g_ref, gp_ref = _oracle(kind, x1, x2, LAM, fe.plan.weights, m.state_dict(),
                                                 fe.pcen.params, tgt.double())
    ef = (feats.detach().double().cpu() - f_ref).abs().max().item()
    ez = rel(z, z_ref)
    names = [n for n, _ in m.named_parameters()]
    g_dev = torch.cat([q.grad.reshape(-1).double().cpu() for q in m.parameters()] +
                      [fe.pcen.params.grad.double().cpu()])
    g_or = torch.cat([g_ref[n].reshape(-1) for n in names] + [gp_ref])
    eg = rel(g_dev, g_or)
    ep = rel(fe.pcen.params.grad, gp_ref)
    print(f"{kind}: features {ef:.2e} logits {ez:.2e} loss {abs(loss.item() - l_ref.item()):.2e} "
          f"arena {eg:.2e} pcen-grad {ep:.2e}")
    assert ef <= 2e-5, ef
    assert ez <= 2e-5, (ez, z, z_ref)
    assert abs(loss.item() - l_ref.item()) <= 2e-5 * max(1.0, abs(l_ref.item()))
    assert eg <= 2e-4, eg
    assert ep <= 1e-3, (ep, fe.pcen.params.grad, gp_ref)

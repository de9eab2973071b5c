"""bf16-operand Winograd F(2x2,3x3) kernels (winograd.hip BF: U images in bf16, V rounded to bf16
(or, with TP_WINO_BF_SPLIT=1, a bf16 hi + lo pair in the MFMA's padding k-slots),
v_mfma_f32_16x16x16_bf16 with fp32 accumulation) against a PyTorch emulation of exactly that
arithmetic and against the fp32 convolution (the bf16 error must be visible, i.e. the bf16 path
really ran)."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

_BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
_G = torch.tensor([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=torch.float64)
_AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def _bf(t):
    return t.float().bfloat16().double()


def _split(v):
    """The BF kernels' V operand: hi = fp32 V truncated to bf16, lo = bf16(V - hi) (round to nearest)."""
    hi = (v.view(torch.int32) & -65536).view(torch.float32)
    return hi.double() + (v - hi).bfloat16().double()


def _wino_bf16_conv(x, w):
    """Emulated BF kernel (V = B^T d B in fp32 as the kernel forms it, rounded to bf16 or split
    into bf16 hi + lo; U in fp64 rounded to bf16; fp64 sums): x (B, H, W, C) NHWC, w (K, C, 3, 3) -> (B, H, W, K) fp64 (even H, W)."""
    B, H, W, C = x.shape
    xp = F.pad(x.permute(0, 3, 1, 2).float(), (1, 1, 1, 1))
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)  # (B, C, H/2, W/2, 4, 4)
    bt = _BT.float()
    V = (bt @ d) @ bt.T  # fp32 in two stages, one rounding per element: the kernel's arithmetic
    V = _split(V) if os.environ.get("TP_WINO_BF_SPLIT") else _bf(V)
    U = _bf(_G @ w.double() @ _G.T)  # (K, C, 4, 4)
    M = torch.einsum("bcyxij,kcij->bkyxij", V, U)
    Y = _AT @ M @ _AT.T  # (B, K, H/2, W/2, 2, 2)
    return Y.permute(0, 2, 4, 3, 5, 1).reshape(B, H, W, -1)


def _epi_fwd(y, scale, shift, pool):
    y = (y * scale.double() + shift.double()).clamp_min(0)
    if pool:
        B, H, W, K = y.shape
        y = y.view(B, H // 2, 2, W // 2, 2, K).amax((2, 4))
    return y


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("K,C", [(32, 8), (64, 96), (256, 40)])
@pytest.mark.parametrize("flip_t", [False, True])
def test_wino_bf16_weights_layout(cuda, K, C, flip_t):
    """bf16 U images == the fp32 images re-laid out (channel pairs packed per dword) and rounded."""
    from torchpruner_amd import ops
    T = ops.require()
    g = torch.Generator().manual_seed(K + C)
    w = torch.randn(C if flip_t else K, K if flip_t else C, 3, 3, generator=g).to(cuda)
    u32 = T.wino_weights(w, flip_t, K, C)
    ubf = T.wino_weights(w, flip_t, K, C, True)
    assert ubf.dtype == torch.bfloat16 and ubf.shape == u32.shape
    # fp32 word ((xi*2 + e)*16 + j)*8 + 2*gs + n; bf16 element 2*((xi*16 + j)*8 + 2*gs + n) + e
    ref = u32.view(C // 8, K // 32, 16, 2, 16, 4, 2).permute(0, 1, 2, 4, 5, 6, 3).reshape(u32.shape)
    assert torch.equal(ubf, ref.bfloat16())


FWD_SHAPES = [(4, 32, 32, 64, 64), (3, 16, 16, 128, 256), (5, 8, 8, 256, 256), (6, 4, 4, 512, 512),
              (3, 14, 14, 64, 64), (2, 28, 28, 32, 64)]


@pytest.mark.parametrize("shape", FWD_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("pool", [False, True])
def test_wino_bf16_fwd(cuda, shape, splits, pool):
    from torchpruner_amd import ops
    T = ops.require()
    B, H, W, C, K = shape
    g = torch.Generator().manual_seed(3 + H * C)
    x = torch.randn(B, H, W, C, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5
    scale = torch.rand(K, generator=g) + 0.5
    shift = torch.randn(K, generator=g) * 0.1
    ubf = T.wino_weights(w.to(cuda), False, K, C, True)
    out, am = T.conv_wino_fwd(x.to(cuda), ubf, scale.to(cuda), shift.to(cuda), True, pool, splits, True)
    emu = _epi_fwd(_wino_bf16_conv(x, w), scale, shift, pool)
    exact = _epi_fwd(F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), padding=1).permute(0, 2, 3, 1),
                     scale, shift, pool)
    assert _rel(out.cpu(), emu) < 2e-5, _rel(out.cpu(), emu)  # the kernel computes what the emulation does
    e = _rel(out.cpu(), exact)
    assert 1e-4 < e < 2e-2, e  # bf16-level error vs the exact conv: the bf16 path ran
    if pool:
        assert am.dtype == torch.uint8


@pytest.mark.parametrize("shape", [(4, 32, 32, 64, 64), (3, 16, 16, 128, 256), (6, 4, 4, 512, 512),
                                   (2, 28, 28, 64, 32)])
@pytest.mark.parametrize("unpool", [False, True])
@pytest.mark.parametrize("splits", [1, 4])
def test_wino_bf16_dgrad(cuda, shape, unpool, splits):
    """Data gradient + Taylor partials with bf16 operands: matches the emulated bf16 conv (the
    transposed, flipped weight) to fp32 accumulation accuracy, including the staged-unpool mode."""
    from torchpruner_amd import ops
    from torchpruner_amd.engine.fused_chain import taylor_slots
    T = ops.require()
    B, H, W, Cin, Cout = shape
    if unpool and not T.wino_staged_ok(H, W, True):
        pytest.skip("no staged-unpool geometry for this map (the engine unpools explicitly there)")
    g = torch.Generator().manual_seed(9 + H * Cin)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * (1.0 / (9 * Cin)) ** 0.5
    act = torch.relu(torch.randn(B, H, W, Cin, generator=g))
    bn_scale = torch.rand(Cin, generator=g) + 0.5
    if unpool:
        gp = torch.randn(B, H // 2, W // 2, Cout, generator=g)
        am = torch.randint(0, 4, (B, H // 2, W // 2, Cout), generator=g, dtype=torch.uint8)
        gfull = torch.zeros(B, H, W, Cout)
        for q in range(4):
            gfull[:, q // 2::2, q % 2::2, :] = torch.where(am == q, gp, torch.zeros(()))
    else:
        gfull = torch.randn(B, H, W, Cout, generator=g)
    wt = w.flip(2, 3).transpose(0, 1).contiguous()  # (Cin, Cout, 3, 3): dgrad = conv(g, wt)
    dx = _wino_bf16_conv(gfull, wt)
    out_emu = torch.where(act > 0, dx * bn_scale.double(), torch.zeros((), dtype=torch.float64))
    tay_emu = (-(dx * act.double())).sum((1, 2))
    ut = T.wino_weights(w.to(cuda), True, Cin, Cout, True)
    R = taylor_slots(H, W)
    tay = torch.zeros(R, B, Cin, device=cuda)
    gin = (gp if unpool else gfull).to(cuda)
    out = T.conv_wino_dgrad(gin, am.to(cuda) if unpool else None, ut, act.to(cuda), bn_scale.to(cuda), tay, True,
                            splits, True)
    assert _rel(out.cpu(), out_emu) < 2e-5, _rel(out.cpu(), out_emu)
    assert _rel(tay.sum(0).cpu(), tay_emu) < 1e-4, _rel(tay.sum(0).cpu(), tay_emu)
    tay2 = torch.zeros_like(tay)
    T.conv_wino_dgrad(gin, am.to(cuda) if unpool else None, ut, act.to(cuda), bn_scale.to(cuda), tay2, True, splits,
                      True)
    assert torch.equal(tay, tay2)  # deterministic


def test_wino_bf16_rejects_direct_mode(cuda):
    from torchpruner_amd import ops
    T = ops.require()
    x = torch.randn(2, 8, 8, 32, device=cuda)
    ubf = T.wino_weights(torch.randn(32, 32, 3, 3, device=cuda), False, 32, 32, True)
    with pytest.raises(RuntimeError):
        T.conv_wino_fwd(x, ubf, None, None, True, False, 1, False)


@pytest.mark.timeout(200)
@pytest.mark.parametrize("variant", ["TP_WINO_BF_K16", "TP_WINO_BF_SPLIT"])
def test_wino_bf16_measured_options_match_emulation(cuda, variant):
    """The launcher reads the option switches once per process, so each option runs the
    emulation check (scripts/probes/wino_bf16_diag.py: 4 VGG shapes, forward) in a child process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **{variant: "1"})
    p = subprocess.run([sys.executable, os.path.join(root, "scripts", "probes", "wino_bf16_diag.py")], env=env, cwd=root,
                       capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rels = [float(ln.split(" rel ")[1].split()[0]) for ln in p.stdout.splitlines() if " rel " in ln]
    assert len(rels) == 4 and max(rels) < 2e-5, p.stdout

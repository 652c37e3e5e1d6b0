"""Large per-GPU batch (288 GB HBM sizing, BASELINE.json config 5): a conv whose output has
more than 2^32 elements.  The epilogue row offsets are 64-bit (csrc/conv_igemm.hip); with
32-bit offsets the images past element 2^32 would wrap onto the first ones.

ResNet-50 stage-1 expansion conv 64 -> 256 at 56x56 with N = 5,400 images: 4.34e9 outputs
(8.7 GB bf16).  Images on both sides of the 2^32 boundary are compared with an fp32 matmul."""
import pytest
import torch

from ddp_classification_pytorch_amd import _ext

pytestmark = pytest.mark.gpu


def test_conv_output_past_2pow32_elements():
    K = _ext.hip_ops()
    N, H, W, Ci, Co = 5400, 56, 56, 64, 256
    assert N * H * W * Co > 2**32
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, Ci, device=dev, generator=g, dtype=torch.float32).bfloat16()
    w = (torch.randn(Co, 1, 1, Ci, device=dev, generator=g) / 8.0).bfloat16()
    y, slabs = K.conv_fwd(x, w, 1, 0, True)
    torch.cuda.synchronize()
    assert y.shape == (N, H, W, Co)
    boundary = 2**32 // (H * W * Co)  # the image holding element 2^32
    for n in (0, boundary - 1, boundary, boundary + 1, N - 1):
        ref = x[n].float().reshape(-1, Ci) @ w.float().reshape(Co, Ci).t()
        got = y[n].float().reshape(-1, Co)
        err = ((got - ref).norm() / ref.norm()).item()
        assert err < 1e-2, (n, err)
    # per-channel statistics from the epilogue cover every row (n = N*H*W)
    st = K.bn_stats(y, slabs)
    assert int(st[0, 0, 0].item()) == N * H * W
    del x, y, slabs
    torch.cuda.empty_cache()


def test_stem_maxpool_past_2pow31_elements():
    """The stem's 3x3/2 max pool at R101 b3072 (BASELINE.json config 5 swept to 3072): the input
    holds 2.47e9 elements, past the old 2^31 flat-index guard; element offsets are 64-bit now."""
    import torch.nn.functional as F

    K = _ext.hip_ops()
    N, H, W, C = 3072, 112, 112, 64
    assert N * H * W * C > 2**31
    dev = torch.device("cuda")
    x = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(1)
    for i in range(0, N, 512):  # fill in chunks: an fp32 temporary of the whole would be 9.9 GB
        x[i:i + 512] = torch.randn(min(512, N - i), H, W, C, device=dev, generator=g).bfloat16()
    y, idx = K.maxpool_fwd(x, 3, 2, 1)
    dy = torch.ones_like(y)
    dx = K.maxpool_bwd(dy, idx, H, W, 3, 2, 1)
    torch.cuda.synchronize()
    for n in (0, 2**31 // (H * W * C), N - 1):
        xn = x[n:n + 1].permute(0, 3, 1, 2).float()
        ref = F.max_pool2d(xn, 3, 2, 1).permute(0, 2, 3, 1)
        assert torch.equal(y[n:n + 1].float(), ref), n
        # every window's argmax receives its 1.0: the gradient mass equals the window count
        assert dx[n].float().sum().item() == float(y[n].numel()), n
    del x, y, idx, dy, dx
    torch.cuda.empty_cache()

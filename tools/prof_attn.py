"""Run the attention kernels at the flagship shape (B32 S256 H8 d64) a few times, for rocprofv3."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparkmi import _native  # noqa: E402


def main():
    C = _native.C()
    B, S, H = 32, 256, 8
    qkv = torch.randn(B, S, 3 * H * 64, device="cuda").bfloat16()
    o = torch.empty(B, S, H * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device="cuda")
    qs = (S * 3 * H * 64, 3 * H * 64, 3 * 64)
    os_ = (S * H * 64, H * 64, 64)
    base = qkv.data_ptr()
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, H, S, device="cuda")
    st = _native.stream()
    for _ in range(int(os.environ.get("ITERS", 10))):
        C.attn_fwd(base, base + 128, base + 256, qs, qs, qs, o.data_ptr(), os_, lse.data_ptr(), 0, B, H, S, S, 1,
                   1.4426950408889634 / 8, st)
        C.attn_bwd(base, base + 128, base + 256, qs, qs, qs, o.data_ptr(), do.data_ptr(), os_, lse.data_ptr(),
                   delta.data_ptr(), dqkv.data_ptr(), dqkv.data_ptr() + 128, dqkv.data_ptr() + 256, 0, B, H, S, S, 1,
                   1.4426950408889634 / 8, 0.125, st)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()

"""The SwiGLU backward of the Llama MLP (T 4096, ffn 14336): dh alone, and dh + dh^T in one
kernel.  Bytes moved
per second.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from collective_communication_mpi_amd.ops import swiglu_pairs_backward  # noqa: E402


def t_us(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


T, k = 4096, 14336
h = torch.randn(T, 2 * k, device="cuda").bfloat16()
da = torch.randn(T, k, device="cuda").bfloat16()
plain = t_us(lambda: swiglu_pairs_backward(h, da))
both = t_us(lambda: swiglu_pairs_backward(h, da, transposed=True))
mb_plain = (T * 2 * k * 2 * 2 + T * k * 2) / 1e6
mb_both = mb_plain + T * 2 * k * 2 / 1e6
print(json.dumps({"dh_us": round(plain, 1), "dh_TBps": round(mb_plain / plain, 2),
                  "dh_and_dht_us": round(both, 1), "dh_and_dht_TBps": round(mb_both / both, 2)}), flush=True)

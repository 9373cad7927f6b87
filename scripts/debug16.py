"""Split-mode checks of the d = 128 kernels at small shapes (debug aid): fused split-KV with
1 / 2 / 4 tiles per split in fp32 and scaled-fp16 partials, and the row-layout partial (O, lse)
against torch fp64."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from exploring_flash_attention_amd import ops  # noqa: E402


def ref(q, k, v):
    s = (q.double() @ k.double().transpose(-1, -2)) / q.shape[-1] ** 0.5
    lse2 = torch.logsumexp(s, -1) / torch.log(torch.tensor(2.0, dtype=torch.float64))
    return torch.softmax(s, -1) @ v.double(), lse2


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    B, H, L, d = 1, 2, 512, 128
    q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    o_ref, lse_ref = ref(q, k, v)
    print("v1", float((ops.attention_v1(q, k, v).double() - o_ref).abs().max()))
    for pd in (torch.float32, torch.bfloat16, ops.PARTIAL_FP16_SCALED):
        for kvt in (1, 2, 4):
            plan = ops.v2_split_plan(B, H, L, d, kvt, q.dtype, blocks_per_workgroup=1)
            o = ops.attention_v2(q, k, v, kvt, partial_dtype=pd, blocks_per_workgroup=1)
            torch.cuda.synchronize()
            print("v2", pd, "kvt", kvt, "plan", plan, "err", float((o.double() - o_ref).abs().max()), flush=True)
    op, lse = ops.attention_partial(q, k, v, partial_dtype=ops.PARTIAL_FP16_SCALED)
    torch.cuda.synchronize()
    lse = lse.reshape(B, H, L, 2)
    e = lse[..., 1].double()
    o_s = op.reshape(B, H, L, d).double() * torch.exp2(e)[..., None]
    print("scaled partial: O err", float((o_s - o_ref).abs().max()), "lse err",
          float((lse[..., 0].double() - lse_ref).abs().max()), "e sample", lse[0, 0, :8, 1].tolist(),
          "row max |O|", o_ref[0, 0, :8].abs().amax(-1).tolist(), "stored max", op.reshape(B, H, L, d)[0, 0, :8].abs().amax(-1).tolist(), flush=True)
    for pd in (torch.float32,):
        op, lse = ops.attention_partial(q, k, v, partial_dtype=pd)
        torch.cuda.synchronize()
        print("partial O err", float((op.reshape(B, H, L, d).double() - o_ref).abs().max()),
              "lse err", float((lse.reshape(B, H, L).double() * 1.0 - (lse_ref + 0)).abs().max()),
              "lse sample", lse.reshape(B, H, L)[0, 0, :4].tolist(), lse_ref[0, 0, :4].tolist(), flush=True)


if __name__ == "__main__":
    main()

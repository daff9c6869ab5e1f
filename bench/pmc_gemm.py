"""Short fixed workload for rocprofv3 PMC passes over the 256²-tile GEMM (profiles/history/r1_pmc_gemm):
3 dispatches each of the schedules in GM_PMC_VARIANTS (default V1,V5) at 8192³, and with
GM_PMC_TORCH=1 three of hipBLASLt's NT kernel on uniform [-1, 1) bf16 operands.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \\
        -d DIR -- python3 bench/pmc_gemm.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gpumounter_amd import _native  # noqa: E402

n = int(os.environ.get("GM_PMC_N", "8192"))
lib = _native.probe()
a = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
bt = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
for v in [int(x) for x in os.environ.get("GM_PMC_VARIANTS", "1,5").split(",")]:
    for _ in range(3):
        assert lib.gm_probe_gemm_nt_variant(v, a.data_ptr(), bt.data_ptr(), c.data_ptr(), n, n, n,
                                            None) == 0
if os.environ.get("GM_PMC_TORCH"):
    for _ in range(3):                       # hipBLASLt NT on the same operands
        torch.matmul(a, bt.t(), out=c)
torch.cuda.synchronize()
print("flops_per_dispatch", 2 * n ** 3)

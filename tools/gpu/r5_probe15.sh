#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp PYTHONPATH=$R; D=gpurun_out/probe15; mkdir -p $D
for v in "attn_only --sync-at 9 --sdpa-math" "both --sync-at 9 --sdpa-math" "attn_only --sync-at 0 --replays 60"; do
  timeout -k 10 240 python -u tools/gpu/bert_graph_nosync.py --variant $v > $D/out.txt 2> $D/err.txt
  rc=$?; echo "rc=$rc $(cut -c1-300 $D/out.txt)"; [ $rc -eq 0 ] || { tail -3 $D/err.txt; exit 1; }
done
python - <<'PY'
import torch, torch.nn.functional as F
from torch.nn.attention import SDPBackend
q = torch.randn(32, 12, 128, 64, device="cuda", requires_grad=True)
for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.MATH):
    try:
        from torch.nn.attention import sdpa_kernel
        with sdpa_kernel([be]):
            F.scaled_dot_product_attention(q, q, q, dropout_p=0.1).sum().backward()
        print("fp32 backend ok:", be)
    except Exception as e:
        print("fp32 backend FAIL:", be, str(e)[:100])
PY

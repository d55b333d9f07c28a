set -o pipefail
timeout -k 10 300 python -u tools/vit_det_probe.py 2>&1 | grep -v "tokens:\|dims:\|heads:\|amdgpu.ids" || exit 1
timeout -k 10 200 python -u tools/determinism_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -u tools/vit_attn_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -u tools/attn_micro.py 2>&1 | grep -v amdgpu.ids | tail -8 || exit 1

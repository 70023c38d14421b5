# hazard fix (v_maximum3 builtin instead of inline-asm v_max3): determinism + numerics + speed
set -o pipefail
O=gpurun_out/r74; mkdir -p $O
timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/fix.so 8 > $O/det_fix.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/base.so abl/fix.so fwd > $O/ab_fix.log 2>&1

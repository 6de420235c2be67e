# Merkle level kernel: parity tests, then the level probe for both kernels
set -o pipefail
out=gpurun_out/${1:-merkle}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "merkle or pointer or combine or pack or c4 or c3_root" tests/test_c4_gpu.py -x -q --timeout 250 --timeout-method thread > $out/tests.log 2>&1 && tail -1 $out/tests.log &&
timeout -k 10 120 python tools/merkle_probe.py > $out/merkle_pc.txt 2>&1 && cat $out/merkle_pc.txt &&
STORMCK_POINTER_RING=3 timeout -k 10 120 python tools/merkle_probe.py > $out/merkle_pc2.txt 2>&1 && cat $out/merkle_pc2.txt &&
STORMCK_POINTER_RING=4 timeout -k 10 120 python tools/merkle_probe.py > $out/merkle_pc3.txt 2>&1 && cat $out/merkle_pc3.txt &&
STORMCK_POINTER_RING=1 timeout -k 10 120 python tools/merkle_probe.py > $out/merkle_ring.txt 2>&1 && cat $out/merkle_ring.txt &&
STORMCK_POINTER_RING=0 timeout -k 10 120 python tools/merkle_probe.py > $out/merkle_quad.txt 2>&1 && cat $out/merkle_quad.txt

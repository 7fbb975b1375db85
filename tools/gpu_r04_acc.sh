set -u
mkdir -p gpurun_out/r04q
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_switch.py -q -k "ws_stagger" --timeout 240 --timeout-method thread > gpurun_out/r04q/switch.out 2>&1 && tail -2 gpurun_out/r04q/switch.out &&
timeout -k 10 200 python tools/gemm_ab.py --only fwd256acc,fwd256 --M 6000000 > gpurun_out/r04q/ab_off.out 2>&1 &&
timeout -k 10 200 env HGIN_WS_STAGGER_ACC=1 python tools/gemm_ab.py --only fwd256acc,fwd256 --M 6000000 > gpurun_out/r04q/ab_on.out 2>&1 &&
cat gpurun_out/r04q/ab_off.out gpurun_out/r04q/ab_on.out

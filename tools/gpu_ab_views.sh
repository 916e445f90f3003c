mkdir -p gpurun_out
AB_VIEWS=16 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C3 base: r56:RT_REFILL=56,RT_COOP=2 r48:RT_REFILL=48,RT_COOP=2 > gpurun_out/ab1.log 2>&1 || exit 1
AB_VIEWS=32 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C3 base: >> gpurun_out/ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab1.log

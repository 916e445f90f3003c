mkdir -p gpurun_out
AB_VIEWS=4 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C4 r24:RT_REFILL=24 r64:RT_REFILL=64 > gpurun_out/ab1.log 2>&1 || exit 1
AB_VIEWS=4 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C2 r24:RT_REFILL=24 r64:RT_REFILL=64 >> gpurun_out/ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab1.log

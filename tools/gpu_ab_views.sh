mkdir -p gpurun_out
AB_VIEWS=1 AB_ROUNDS=5 timeout -k 10 300 python tools/ab_views.py C3 base: r64c2:RT_REFILL=64,RT_COOP=2 r40c2:RT_REFILL=40,RT_COOP=2 > gpurun_out/ab1.log 2>&1 || exit 1
AB_VIEWS=4 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C4 base: coop2:RT_COOP=2 >> gpurun_out/ab1.log 2>&1 || exit 1
AB_VIEWS=1 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C4 base: r64c2:RT_REFILL=64,RT_COOP=2 >> gpurun_out/ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab1.log

mkdir -p gpurun_out
AB_VIEWS=8 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C2 base: df:RT_KERNEL=df > gpurun_out/ab1.log 2>&1 || exit 1
AB_VIEWS=2 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C5 base: df:RT_KERNEL=df >> gpurun_out/ab1.log 2>&1 || exit 1
AB_VIEWS=1 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C5 base: df:RT_KERNEL=df df64:RT_KERNEL=df,RT_REFILL=64,RT_COOP=2 >> gpurun_out/ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab1.log

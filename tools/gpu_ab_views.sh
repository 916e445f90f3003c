mkdir -p gpurun_out
AB_VIEWS=16 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C3 base: r48:RT_REFILL=48 wpe1:RT_WPE=1 nocoop:RT_COOP=0 noxcd:RT_XCD=0 > gpurun_out/ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab1.log

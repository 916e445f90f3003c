mkdir -p gpurun_out
AB_VIEWS=16 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_views.py C3 base: wpe3:RT_WPE=3 wpe4:RT_WPE=4 > gpurun_out/ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab1.log

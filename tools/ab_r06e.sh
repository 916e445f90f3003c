# developer A/B of library builds (run on the GPU box): LIBS (build/*.so names) x CFGS (cfg:views:rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in ${LIBS:-base_librt lib_RT_PLANES_U81}; do
  for c in ${CFGS:-C3:64:3 C4:16:2 C5:1:2}; do
    IFS=: read -r cfg v r <<< "$c"
    timeout -k 10 300 python -u tools/ab_variants.py $cfg --views $v --rounds $r --arms x: --lib raytracer-group27_amd/build/$lib.so > gpurun_out/ab_${TAG:-r06e}_${cfg}_$lib.log 2>&1 || exit 1
    echo "$lib $(tail -1 gpurun_out/ab_${TAG:-r06e}_${cfg}_$lib.log)"
  done
done

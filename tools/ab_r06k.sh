# developer A/B (run on the GPU box): the in-tree library (every automatic variable defined) against
# build/base_librt.so (without), C3 / C4 / C5, and the 4-wave recursion-tree build (RT_OPT_TREE 4) on C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for lib in base new; do
  L=""; [ $lib = base ] && L="--lib raytracer-group27_amd/build/base_librt.so"
  A="x:"; [ $lib = new ] && A="x: tree4:13=4"
  for c in C3:64:3 C4:16:2 C5:1:2; do
    IFS=: read -r cfg v r <<< "$c"
    arms="x:"; [ $cfg != C3 ] && arms="$A"
    timeout -k 10 300 python -u tools/ab_variants.py $cfg --views $v --rounds $r --arms $arms $L > gpurun_out/ab_r06k_${cfg}_${lib}_$rep.log 2>&1 || exit 1
    grep "ms" gpurun_out/ab_r06k_${cfg}_${lib}_$rep.log | sed "s/^/$lib /" | cut -c1-200
  done
done
done

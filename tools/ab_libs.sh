set -o pipefail
for lib in new base; do
  L=""; [ $lib = base ] && L="--lib raytracer-group27_amd/build/base_librt.so"
  timeout -k 10 300 python -u tools/ab_variants.py C3 --views 64 --rounds 3 --arms op: cm4:3=4 $L > gpurun_out/ab_${TAG}_C3_$lib.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_variants.py C4 --views 16 --rounds 2 --arms d: $L > gpurun_out/ab_${TAG}_C4_$lib.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_variants.py C5 --views 2 --rounds 2 --arms d: $L > gpurun_out/ab_${TAG}_C5_$lib.log 2>&1 || exit 1
done
grep -h "ms" gpurun_out/ab_${TAG}_*.log

mkdir -p gpurun_out/ab
for r in 1 2; do for sk in 0 16896 4608 66048; do
MSPLIT_BASIS_SKEW=$sk timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/ab/skew_${sk}_$r.json 2>/dev/null || exit 1
done; done

cd $GRAFT_REPO_ROOT
for L in 2 4 8 16 24; do
  echo "lead=$L $(WG_K1_LEAD=$L timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2>/dev/null | grep -o '"kernel_ms": {[^}]*}')" || exit 1
done
echo "default $(timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2>/dev/null | grep -o '"kernel_ms": {[^}]*}')"

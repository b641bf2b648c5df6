# bench order: breakdown pass before the warmup iterations (new default) vs after (--breakdown-last), driver shape
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p15
mkdir -p $O
cd $R
B() { n=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; exit 1; }; }
B first1 && B last1 --breakdown-last && B first2 && B last2 --breakdown-last && B first3 && B last3 --breakdown-last
echo "rc=$?"

# Round 6: smoke() and the default bench of the shipped library (reads the
# r06_ay PMC summaries recorded for it).
# usage (on the box): bash probes/g_r06ba.sh SET
set -e
S=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$S
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1

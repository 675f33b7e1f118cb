# round 6 call g: side-stream x update with per-solve events (host overhead cut): mv_ab alternated, and a kernel trace
# of the side mode's CG loop (is k_axpy_dev beside k_render_matvec?)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for m in 0 1; do
    GSLM_CG_SIDE_X=$m timeout -k 10 240 python tools/mv_ab.py side$m --reps 30 --out /tmp/gslm_ab > $O/mv_side${m}_r$r.json 2> $O/mv_side${m}_r$r.err || { tail -5 $O/mv_side${m}_r$r.err; exit 1; }
    cat $O/mv_side${m}_r$r.json
  done
done
ROOT=$(pwd)
(cd /tmp && GSLM_CG_SIDE_X=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $ROOT/$O/trace -o run -- python3 $ROOT/tools/mv_ab.py side1 --reps 10 --out /tmp/gslm_ab > $ROOT/$O/trace.json 2> $ROOT/$O/trace.err) || { tail -5 $O/trace.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r06g/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if any(k in r["Kernel_Name"] for k in ("k_render_matvec<false>", "k_axpy_dev", "k_preprocess_jvp", "k_gather_lm", "k_cg_update"))]
t0 = int(ks[-60]["Start_Timestamp"])
for r in ks[-40:]:
    print(f'{r["Kernel_Name"][:40]:40s} q{r.get("Queue_Id","?"):>3s} start {(int(r["Start_Timestamp"])-t0)/1000:9.1f} dur {(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000:7.1f}')
PY

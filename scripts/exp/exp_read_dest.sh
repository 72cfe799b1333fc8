# Experiment driver: write the config-1 directory, list it, run the read
# destination experiments (C host with /opt/rocm's runtime; host-only binary
# with each runtime dlopen'ed).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
D=$(mktemp -d /tmp/rd_XXXXXX)
python3 -c "
import sys; sys.path.insert(0, '.')
from spacedrive_amd import corpus
paths, sizes = corpus.write_config1_dir('$D/c1', 10000, seed=1)
open('$D/list.txt', 'w').write(''.join(f'{p} {int(s)}\n' for p, s in zip(paths, sizes)))
" || exit 1
TL=$(python3 -c "import torch, os; print(os.path.dirname(torch.__file__) + '/lib/libamdhip64.so')")
timeout -k 10 300 ./build/exp_read_dest $D/list.txt > gpurun_out/${TAG}_readdest.log 2>&1 || exit 1
timeout -k 10 300 ./build/exp_read_dest_dl $D/list.txt /opt/rocm/lib/libamdhip64.so.7 >> gpurun_out/${TAG}_readdest.log 2>&1 || exit 1
timeout -k 10 300 ./build/exp_read_dest_dl $D/list.txt $TL >> gpurun_out/${TAG}_readdest.log 2>&1 || exit 1
rm -rf $D
echo "exit 0"

set -o pipefail
mkdir -p gpurun_out/r47
python3 -c "
import sys; sys.path.insert(0,'.')
from broadway_amd import gen
open('/tmp/s.h264','wb').write(gen.generate(3,100))
"
S=broadway_amd/csrc
for v in old new; do
  if [ $v = old ]; then D=gpurun_out/r47/oldsrc; mkdir -p $D; tar -xf tools/oldsrc.tar -C $D; SS=$D/broadway_amd/csrc; else SS=$S; fi
  gcc -O3 -std=gnu11 -I$SS tools/ubench/parse_cpu.c $SS/common/*.c $SS/host/syntax.c $SS/host/slicedata.c $SS/host/dpb.c $SS/host/decoder.c $SS/host/conceal.c $SS/host/specparse.c $SS/host/capture.c -lpthread -lm -o /tmp/pc_$v || exit 1
done
for i in 1 2; do for v in old new; do echo -n "$v threads1 "; H264MI_PARSE_THREADS=1 timeout 120 /tmp/pc_$v /tmp/s.h264; echo -n "$v threads4 "; H264MI_PARSE_THREADS=4 timeout 120 /tmp/pc_$v /tmp/s.h264; done; done

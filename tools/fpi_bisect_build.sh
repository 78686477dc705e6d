#!/bin/bash
# Builds the three engine variants tools/fpi_bisect.sh compares, from the tree as it was before
# commit 085e3ba (git worktree in /tmp), into tools/_bisect/{A,B,C} (git-ignored).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/edgpu_r01old
rm -rf $W; git -C $R worktree add -f $W 085e3ba^ -q
E=$W/easydarwin_amd/csrc/edgpu_engine.cpp
cp $E /tmp/edgpu_engine_A.cpp
python3 - <<'PY'
s = open('/tmp/edgpu_engine_A.cpp').read()
b = s.replace("""        HIP_CHECK(hipMemcpyAsync(x->d_blob, blob, blob_bytes, hipMemcpyHostToDevice, x->stream));
        dd = x->d_desc;""", """        HIP_CHECK(hipMemcpyAsync(x->d_blob, blob, blob_bytes, hipMemcpyHostToDevice, x->stream));
        HIP_CHECK(hipStreamSynchronize(x->stream));
        dd = x->d_desc;""", 1)
c = s.replace("""    HIP_CHECK(hipMallocAsync((void**)&dq, q.size() * sizeof(FirstInfoQuery), x->stream));
    HIP_CHECK(hipMallocAsync((void**)&dr, q.size() * sizeof(FirstInfoResult), x->stream));""",
              """    HIP_CHECK(hipMalloc((void**)&dq, q.size() * sizeof(FirstInfoQuery)));
    HIP_CHECK(hipMalloc((void**)&dr, q.size() * sizeof(FirstInfoResult)));""", 1)
c = c.replace("""    HIP_CHECK(hipFreeAsync(dq, x->stream));
    HIP_CHECK(hipFreeAsync(dr, x->stream));
    HIP_CHECK(hipStreamSynchronize(x->stream));""", """    HIP_CHECK(hipStreamSynchronize(x->stream));
    HIP_CHECK(hipFree(dq));
    HIP_CHECK(hipFree(dr));""", 1)
assert b != s and c != s
open('/tmp/edgpu_engine_B.cpp', 'w').write(b)
open('/tmp/edgpu_engine_C.cpp', 'w').write(c)
# D = B + C: ingest waits, RTP-Info buffers from hipMalloc
d = b.replace("""    HIP_CHECK(hipMallocAsync((void**)&dq, q.size() * sizeof(FirstInfoQuery), x->stream));
    HIP_CHECK(hipMallocAsync((void**)&dr, q.size() * sizeof(FirstInfoResult), x->stream));""",
              """    HIP_CHECK(hipMalloc((void**)&dq, q.size() * sizeof(FirstInfoQuery)));
    HIP_CHECK(hipMalloc((void**)&dr, q.size() * sizeof(FirstInfoResult)));""", 1)
d = d.replace("""    HIP_CHECK(hipFreeAsync(dq, x->stream));
    HIP_CHECK(hipFreeAsync(dr, x->stream));
    HIP_CHECK(hipStreamSynchronize(x->stream));""", """    HIP_CHECK(hipStreamSynchronize(x->stream));
    HIP_CHECK(hipFree(dq));
    HIP_CHECK(hipFree(dr));""", 1)
# F = B + pinned host query / result staging, pool device buffers kept
f = b.replace("""    HIP_CHECK(hipMemcpyAsync(dq, q.data(), q.size() * sizeof(FirstInfoQuery), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(launch_first_packet_info(dq, dr, x->d_senders.ptr, sh.ntracks, x->stream));
    HIP_CHECK(hipMemcpyAsync(r.data(), dr, r.size() * sizeof(FirstInfoResult), hipMemcpyDeviceToHost, x->stream));
    HIP_CHECK(hipFreeAsync(dq, x->stream));
    HIP_CHECK(hipFreeAsync(dr, x->stream));
    HIP_CHECK(hipStreamSynchronize(x->stream));""", """    static FirstInfoQuery* hq = nullptr;
    static FirstInfoResult* hr = nullptr;
    if (!hq) { HIP_CHECK(hipHostMalloc((void**)&hq, 64 * sizeof(FirstInfoQuery), 0));
               HIP_CHECK(hipHostMalloc((void**)&hr, 64 * sizeof(FirstInfoResult), 0)); }
    memcpy(hq, q.data(), q.size() * sizeof(FirstInfoQuery));
    HIP_CHECK(hipMemcpyAsync(dq, hq, q.size() * sizeof(FirstInfoQuery), hipMemcpyHostToDevice, x->stream));
    HIP_CHECK(launch_first_packet_info(dq, dr, x->d_senders.ptr, sh.ntracks, x->stream));
    HIP_CHECK(hipMemcpyAsync(hr, dr, r.size() * sizeof(FirstInfoResult), hipMemcpyDeviceToHost, x->stream));
    HIP_CHECK(hipFreeAsync(dq, x->stream));
    HIP_CHECK(hipFreeAsync(dr, x->stream));
    HIP_CHECK(hipStreamSynchronize(x->stream));
    memcpy(r.data(), hr, r.size() * sizeof(FirstInfoResult));""", 1)
# Bi = B + a second, synchronous read of the result and query buffers before they are freed
bi = b.replace("""    HIP_CHECK(hipMemcpyAsync(r.data(), dr, r.size() * sizeof(FirstInfoResult), hipMemcpyDeviceToHost, x->stream));
    HIP_CHECK(hipFreeAsync(dq, x->stream));
    HIP_CHECK(hipFreeAsync(dr, x->stream));
    HIP_CHECK(hipStreamSynchronize(x->stream));""", """    HIP_CHECK(hipMemcpyAsync(r.data(), dr, r.size() * sizeof(FirstInfoResult), hipMemcpyDeviceToHost, x->stream));
    HIP_CHECK(hipStreamSynchronize(x->stream));
    {
        std::vector<FirstInfoResult> r2(sh.ntracks);
        std::vector<FirstInfoQuery> q2(sh.ntracks);
        HIP_CHECK(hipMemcpy(r2.data(), dr, r2.size() * sizeof(FirstInfoResult), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(q2.data(), dq, q2.size() * sizeof(FirstInfoQuery), hipMemcpyDeviceToHost));
        for (uint32_t t = 0; t < sh.ntracks; t++)
            fprintf(stderr, "FPI now=%lld t=%u first=%u,%u reread=%u,%u query_ok=%d dq=%p dr=%p\\n", (long long)now_ms, t,
                    r[t].found, r[t].seq, r2[t].found, r2[t].seq,
                    memcmp(&q2[t], &q[t], sizeof(FirstInfoQuery)) == 0, (void*)dq, (void*)dr);
    }
    HIP_CHECK(hipFreeAsync(dq, x->stream));
    HIP_CHECK(hipFreeAsync(dr, x->stream));
    HIP_CHECK(hipStreamSynchronize(x->stream));""", 1)
assert d != b and f != b and bi != b
open('/tmp/edgpu_engine_D.cpp', 'w').write(d)
open('/tmp/edgpu_engine_F.cpp', 'w').write(f)
open('/tmp/edgpu_engine_Bi.cpp', 'w').write(bi)
PY
for v in A B C D F Bi; do
  cp /tmp/edgpu_engine_$v.cpp $E
  make -C $W/easydarwin_amd/csrc -s -B
  mkdir -p $R/tools/_bisect/$v/easydarwin_amd $R/tools/_bisect/$v/tools
  cp $W/easydarwin_amd/libedgpu.so $R/tools/_bisect/$v/easydarwin_amd/
  cp $W/tools/adapter_replay $R/tools/_bisect/$v/tools/
done
(cd $W && python3 -c "
import sys, json
sys.path[:0] = ['.', 'tests']
from scenarios import SCENARIOS
SCENARIOS['rtpinfo']().write('$R/tools/_bisect/rtpinfo.edtr')
print(json.load(open('tests/golden/rtpinfo.json'))['capture_sha256'])") > $R/tools/_bisect/rtpinfo.sha
git -C $R worktree remove --force $W

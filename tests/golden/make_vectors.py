"""Regenerates the cold-path parser vectors in tests/golden/ from the REAL reference.

* sdp_vectors.json -- SDP texts (edge cases of the m= / a=rtpmap / a=control parse) and, per
  stream, what SDPSourceInfo::Parse (APICommonCode/SDPSourceInfo.cpp:172-420) makes of them:
  payload type, payload name (compared byte for byte by the H.264 keyframe gate,
  ReflectorStream.cpp:1879), trackID, port, TCP flag.
* keyframecache_vectors.json -- op scripts over CKeyFrameCache (CommonUtilitiesLib/
  keyframecache.cpp:6-118): PutOnePacket (TLV [0x28][BE16 len][bytes][0x29] through the 5 KiB
  scratch, the buf[13] rewrite, the SPS reset), GetOnePacket (STX / length / ETX checks),
  SetBuf (mem_size overflow); per op the result, the caller's buffer after the call and
  curdatalen.  Cases where the reference itself is undefined (PutOnePacket with len > 5116
  overruns its stack scratch -- FrameBuffer::Encode ignores the capacity; start == 1 with
  len < 14 writes past the packet) are left out: they are the restatement's own documented
  choices (refuse / skip the rewrite), tested in tests/test_cold_parsers.py without a pin.

Runs oracle/_ref/ref_vectors (the reference sources compiled by oracle/_ref/Makefile) in a
scratch directory (PutOnePacket appends to ./data.264).  Run here: python tests/golden/make_vectors.py
The output files are data (inputs + the reference's outputs).
"""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from easydarwin_amd.synth import TrackSpec, make_sdp  # noqa: E402


def sdp_cases() -> list[bytes]:
    base = make_sdp([TrackSpec("video", "H264/90000", 96), TrackSpec("audio", "PCMA/8000", 8)]).encode()
    c = [
        base,
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=rtpmap:96 h264/90000\r\n",                  # lowercase
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=rtpmap:96 H264/90000  \r\n",                # trailing spaces
        b"v=0\r\nm=video 0 RTP/AVP 96 97\r\na=rtpmap:96 H264/90000\r\na=rtpmap:97 H265/90000\r\n",
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=rtpmap:96\r\na=rtpmap:96 H264/90000\r\n",   # first rtpmap without name
        b"v=0\r\na=rtpmap:96 H264/90000\r\nm=video 0 RTP/AVP 96\r\n",                  # rtpmap before m=
        b"v=0\r\nm=application 0 RTP/AVP 107\r\na=rtpmap:107 vnd.onvif.metadata/90000\r\n"
        b"m=video 0 RTP/AVP 96\r\na=rtpmap:96 H264/90000\r\n",
        b"v=0\r\nm=video 5004 RTP/AVP/TCP 96\r\na=rtpmap:96 H264/90000\r\n",
        b"v=0\nm=video 0 RTP/AVP 96\na=rtpmap:96 H264/90000\nm=audio 0 RTP/AVP 0\na=rtpmap:0 PCMU/8000\n",
        b"v=0\rm=video 0 RTP/AVP 96\ra=rtpmap:96 H264/90000\r",                           # CR only
        b"v=0\r\n\r\n\r\nm=video 0 RTP/AVP 96\r\n\n\na=rtpmap:96 H264/90000\r\n\r\n",     # blank lines
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=control:trackID=3\r\na=rtpmap:96 H264/90000\r\n"
        b"m=audio 0 RTP/AVP 8\r\na=control:trackID=1\r\na=rtpmap:8 PCMA/8000\r\n",       # trackIDs out of order
        b"v=0\r\na=control:*\r\nm=video 0 RTP/AVP 96\r\na=control:*\r\nm=audio 0 RTP/AVP 8\r\n"
        b"a=control:rtsp://10.0.0.1:554/live/x.sdp/trackID=7\r\nm=audio 0 RTP/AVP 0\r\na=control:track5\r\n"
        b"m=video 0 RTP/AVP 96\r\na=control:streamid=12\r\n",
        b"v=0\r\nm=video\t0 RTP/AVP 96\r\na=rtpmap:96 H264/90000\r\nmvideo 0\r\nm=VIDEO 0 RTP/AVP 96\r\n"
        b"m=video2 0 RTP/AVP 96\r\nm=audio_x 0\r\n",
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=rtpmap 96 H264/90000\r\n",                   # no colon
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=rtpmap:96 H264/90000/1\r\n",
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=RTPMAP:96 H264/90000\r\na=rtpmap:96 MP4V-ES/90000\r\n",
        b"v=0\r\ns=no media\r\n",
        b"",
        b"v=0\r\nm=audio 0 RTP/AVP 97\r\na=rtpmap:97 MPEG4-GENERIC/48000/2\r\na=fmtp:97 streamtype=5\r\n"
        b"m=video 0 RTP/AVP 26\r\na=rtpmap:26 JPEG/90000\r\n",
        b"v=0\r\nm=video 0 RTP/AVP 96\r\na=rtpmap:96   H264/90000\r\n",                # several spaces
        b"v=0\r\nm=\r\nm\r\na=rtpmap:96 X/1\r\n",
    ]
    c.append(b"v=0\r\n" + b"".join(b"m=audio 0 RTP/AVP 0\r\na=rtpmap:0 PCMU/8000\r\n" for _ in range(16)))
    return c


def kfc_scripts() -> list[list[tuple]]:
    """Op scripts: (code, a, b, bytes); 0 new(len=a), 1 put(nalutype=a, start=b), 2 get(offset=a),
    3 setbuf."""
    def pkt(n, seed):
        return bytes(((i * 37 + seed * 11) & 0xFF) for i in range(n))
    s1 = [(0, 2 << 20, 0, b""),
          (1, 7, 1, pkt(30, 1)), (1, 8, 1, pkt(20, 2)), (1, 5, 1, pkt(1400, 3)), (1, 5, 0, pkt(1400, 4)),
          (1, 1, 1, pkt(900, 5)), (1, 1, 0, pkt(14, 6)),
          (2, 0, 0, b""), (2, 34, 0, b""), (2, 58, 0, b""), (2, 1462, 0, b""), (2, 2866, 0, b""),
          (2, 1, 0, b""), (2, 3860, 0, b""),
          (1, 7, 1, pkt(40, 7)), (2, 0, 0, b""), (2, 44, 0, b""),             # SPS resets curdatalen
          (1, 5, 1, pkt(5116, 8)), (2, 44, 0, b""),                             # the 5 KiB scratch, full
          (1, 5, 1, b""), (3, 0, 0, b""),                                       # empty: refused
          (1, 9, 0, pkt(3, 9)), (1, 9, 0, pkt(1, 10))]
    s2 = [(0, 100, 0, b""),                                                     # mem_size overflow
          (1, 1, 0, pkt(40, 11)), (1, 1, 0, pkt(40, 12)), (1, 1, 0, pkt(12, 13)), (1, 1, 0, pkt(11, 14)),
          (3, 0, 0, bytes([1])), (3, 0, 0, bytes([2, 3])),
          (2, 0, 0, b""), (2, 44, 0, b""), (2, 88, 0, b""), (2, 99, 0, b""), (2, 100, 0, b"")]
    s3 = [(0, 4096, 0, b""),                                                    # crafted records
          (3, 0, 0, bytes([0x28, 0x00, 0x02, 0x61, 0x62, 0x29])),               # good
          (3, 0, 0, bytes([0x28, 0x00, 0x02, 0x61, 0x62, 0x00])),               # bad ETX
          (3, 0, 0, bytes([0x27, 0x00, 0x01, 0x61, 0x29])),                     # bad STX
          (3, 0, 0, bytes([0x28, 0x00, 0x00, 0x29])),                           # empty record
          (3, 0, 0, bytes([0x28, 0xFF, 0xFF, 0x00] + [0] * 12)),                # length >= curdatalen
          (2, 0, 0, b""), (2, 6, 0, b""), (2, 12, 0, b""), (2, 17, 0, b""), (2, 21, 0, b""),
          (1, 7, 1, pkt(16, 15)), (2, 0, 0, b"")]
    return [s1, s2, s3]


def pack_cases(cases):
    return struct.pack("<I", len(cases)) + b"".join(struct.pack("<I", len(c)) + c for c in cases)


def pack_script(ops):
    out = [struct.pack("<I", len(ops))]
    for code, a, b, data in ops:
        out.append(struct.pack("<BiiI", code, a, b, len(data)) + data)
    return b"".join(out)


def main():
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_vectors")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    with tempfile.TemporaryDirectory() as td:
        cases = sdp_cases()
        p = os.path.join(td, "sdp.bin")
        open(p, "wb").write(pack_cases(cases))
        out = json.loads(subprocess.run([exe, "sdp", p], capture_output=True, check=True, cwd=td).stdout)
        vec = [{"sdp_hex": c.hex(), "streams": o} for c, o in zip(cases, out)]
        json.dump({"source": "oracle/_ref/ref_vectors sdp (SDPSourceInfo::Parse of the reference)",
                   "generator": "tests/golden/make_vectors.py", "cases": vec},
                  open(os.path.join(HERE, "sdp_vectors.json"), "w"), indent=1)
        scripts = []
        for k, ops in enumerate(kfc_scripts()):
            p = os.path.join(td, f"kfc{k}.bin")
            open(p, "wb").write(pack_script(ops))
            res = json.loads(subprocess.run([exe, "kfc", p], capture_output=True, check=True, cwd=td).stdout)
            scripts.append({"ops": [[c, a, b, d.hex()] for c, a, b, d in ops], "results": res})
        json.dump({"source": "oracle/_ref/ref_vectors kfc (CKeyFrameCache of the reference)",
                   "generator": "tests/golden/make_vectors.py", "scripts": scripts},
                  open(os.path.join(HERE, "keyframecache_vectors.json"), "w"), indent=1)
    print(f"{len(cases)} SDP cases, {len(scripts)} keyframecache scripts")


if __name__ == "__main__":
    main()

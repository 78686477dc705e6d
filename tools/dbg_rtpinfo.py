import sys, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from scenarios import SCENARIOS
from easydarwin_amd import edgpu
from easydarwin_amd.trace import JOIN, PKT, TICK
tr = SCENARIOS['rtpinfo']()
ctx = edgpu.Context()
for sdp in tr.sdps: ctx.session_add(sdp)
pending=[]; clock=0; handles={}
def flush():
    global pending
    if pending:
        ctx.ingest_host(*edgpu.build_batch(pending)); ctx.keyframe_index(); pending=[]
joins=[]
out=open(sys.argv[1],'w')
for ev in tr.events:
    clock=max(clock, ev[1])
    if ev[0]==PKT: pending.append((ev[2],ev[3],ev[1],ev[4]))
    elif ev[0]==JOIN:
        if ev[5]&1: flush()
        joins.append(ev+(clock,))
    else:
        flush()
        for (_,jt,s,sub,trn,ua,nj) in joins:
            try:
                h,info=ctx.subscriber_play(s, trn, bool(ua&1), nj); handles[h]=sub
                print('join', sub, 'h', h, 'info', info, 'now', nj, file=out)
            except edgpu.EdgpuError as e:
                print('deferred', sub, e, file=out)
        joins=[]
        r=ctx.fanout(ev[1]); st,subs,desc,arena=ctx.read_tick(r)
        for q in subs:
            if handles.get(int(q['subscriber'])) in (20,21,22,23) and q['desc_count']:
                d=desc[int(q['desc_base']):int(q['desc_base'])+int(q['desc_count'])]
                print('tick', ev[1], 'sub', handles[int(q['subscriber'])], 'kind', int(q['kind']), 'n', int(q['desc_count']), 'ids', int(d['packet_id'][0]), int(d['packet_id'][-1]), file=out)
out.close()

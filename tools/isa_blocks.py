import re,sys
lines=open(sys.argv[1]).read().split('\n')
a,b=int(sys.argv[2]),int(sys.argv[3])
blk=None;cnt={}
order=[]
for l in lines[a-1:b]:
    m=re.match(r'^(\.LBB\d+_\d+|; %bb\.\d+):',l)
    if m:
        blk=m.group(1);order.append(blk);cnt[blk]={'v':0,'s':0,'ds':0,'g':0,'vm':0};continue
    t=l.strip().split()
    if not t or t[0].startswith(';') or t[0].startswith('.'): continue
    op=t[0]
    c=cnt.setdefault(blk,{'v':0,'s':0,'ds':0,'g':0,'vm':0})
    if op.startswith('v_'):
        c['v']+=1
        if op.startswith('v_mov'): c['vm']+=1
    elif op.startswith('s_'): c['s']+=1
    elif op.startswith('ds_'): c['ds']+=1
    elif op.startswith('global_') or op.startswith('flat_') or op.startswith('buffer_'): c['g']+=1
for k in order: print(k, cnt[k])
print('total', {x:sum(c[x] for c in cnt.values()) for x in ['v','s','ds','g','vm']})

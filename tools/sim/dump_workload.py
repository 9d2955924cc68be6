import sys, numpy as np
import os as _os
_root = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
sys.path.insert(0, _root); sys.path.insert(0, _os.path.join(_root, 'oracle'))
import oracle as O
from openwhisk_amd import workload as W
name = sys.argv[1]; nact = int(sys.argv[2]) if len(sys.argv)>2 else None
out_root = sys.argv[3] if len(sys.argv) > 3 else '/tmp/sim'
ns = int(sys.argv[4]) if len(sys.argv) > 4 else 1
w = W.config(name, n_activations=nact, n_shards=ns)
if ns > 1: name = f'{name}_of{ns}'
st = O.state_for(w)
nm, nb = st.managed_size, st.blackbox_size
ms, bs = np.array(st.managed_step_sizes,np.int32), np.array(st.blackbox_step_sizes,np.int32)
n = len(w.inv_ids)
ids = w.inv_ids
usable = (w.inv_status==0)
mpool = ids[:nm]; bpool = ids[n-nb:]
A = len(w.actions)
keys = {}
home=np.zeros(A,np.int32); step=np.zeros(A,np.int32); mem=np.zeros(A,np.int32); maxc=np.zeros(A,np.int32); pool=np.zeros(A,np.int32); slot=np.zeros(A,np.int32)
for i,a in enumerate(w.actions):
    h = st.action_hash(i)
    p = 1 if a.blackbox else 0
    nn = nb if p else nm; ss = bs if p else ms
    home[i] = h % nn; step[i] = ss[h % len(ss)] % nn
    mem[i]=a.mem_mb; maxc[i]=a.max_concurrent; pool[i]=p; slot[i]=keys.setdefault(a.key,len(keys))
perm = st.permits()
out, fl, rf = st.replay(w.stream)
s = w.stream
import os
os.makedirs(out_root, exist_ok=True)
np.savez(f'{out_root}/{name}.npz', perm=perm, mpool=mpool.astype(np.int32), bpool=bpool.astype(np.int32), usable=usable.astype(np.int32),
  home=home, step=step, mem=mem, maxc=maxc, pool=pool, slot=slot, act=s.act.astype(np.int32), acq_off=s.acq_off, rel_off=s.rel_off, rel_aid=s.rel_aid,
  out=out, fl=fl, rf=rf, seed=np.array([w.rng_seed],np.uint64))
print(name, n, nm, nb, A, len(s.act), s.n_batches, len(s.rel_aid), 'fallbacks', int((fl&1).sum()), 'perm0', perm[:3])
import os
d=f'{out_root}/{name}'; os.makedirs(d, exist_ok=True)
for k,v in dict(perm=perm.astype(np.int32), mpool=mpool.astype(np.int32), bpool=bpool.astype(np.int32), usable=usable.astype(np.int32),
  home=home, step=step, mem=mem, maxc=maxc, pool=pool, slot=slot, act=s.act.astype(np.int32), acq_off=s.acq_off.astype(np.int64), rel_off=s.rel_off.astype(np.int64), rel_aid=s.rel_aid.astype(np.int64),
  out=out.astype(np.int32), fl=fl.astype(np.uint8), seed=np.array([w.rng_seed],np.uint64)).items():
    v.tofile(f'{d}/{k}.bin')

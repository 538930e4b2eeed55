import ctypes as C, sys, os
sys.path[:0] = ['tests', 'oracle']
import numpy as np
import refcpu
from devbuf import Dev
from refapi import mq
lib = mq.load(); mq.check(lib.mq_init(0))
n = 1 << 16
a, b, p = refcpu.gen_join(n, 'build'), refcpu.gen_join(n, 'probe'), refcpu.gen_join(n, 'iota')
w1, w2 = refcpu.hash_join(a, p, b, p)
def run(c1, p1, c2, p2):
    D = [Dev.of(x) for x in (c1, p1, c2, p2)]
    h = C.c_void_p(); mq.check(lib.mq_join_build(D[0].ptr, D[1].ptr, len(c1), C.byref(h), None))
    m = C.c_uint64(); mq.check(lib.mq_join_probe(h, D[2].ptr, len(c2), C.byref(m), None)); m = m.value
    o1, o2 = Dev(m * 4 + 4), Dev(m * 4 + 4)
    mq.check(lib.mq_join_write(h, D[3].ptr, o1.ptr, o2.ptr, None))
    mq.check(lib.mq_stream_sync(None))
    r = o1.get(np.int32, m), o2.get(np.int32, m)
    mq.check(lib.mq_join_free(h))
    return r
g1, g2 = run(a, p, b, p)
print('M', len(g1), len(w1))
bad = np.nonzero((g1 != w1) | (g2 != w2))[0]
print('mismatches', len(bad), bad[:10])
for i in bad[:5]:
    print(i, 'got', g1[i], g2[i], 'want', w1[i], w2[i], 'keys', a[w1[i]], b[w2[i]], a[g1[i]] if 0 <= g1[i] < n else None)
# device-generated inputs
Dd = {k: Dev(n * 4) for k in 'abp'}
mq.check(lib.mq_gen_join_keys(Dd['a'].ptr, n, 0, None)); mq.check(lib.mq_gen_join_keys(Dd['b'].ptr, n, 1, None)); mq.check(lib.mq_gen_iota(Dd['p'].ptr, n, None))
for k, ref in (('a', a), ('b', b), ('p', p)):
    print('gen', k, np.array_equal(Dd[k].get(np.int32, n), ref))
rng = np.random.default_rng(1)
x = rng.integers(-(2**31), 2**31 - 1, 30000, dtype=np.int64).astype(np.int32)
c1 = np.concatenate([x, x[:5000], x[100:200]]); c2 = np.concatenate([x[::7], rng.integers(-9, 9, 100).astype(np.int32)])
p1 = np.arange(len(c1), dtype=np.int32); p2 = np.arange(len(c2), dtype=np.int32) + 7
g1, g2 = run(c1, p1, c2, p2); w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
print('wide dups equal', np.array_equal(g1, w1) and np.array_equal(g2, w2), len(g1), len(w1))

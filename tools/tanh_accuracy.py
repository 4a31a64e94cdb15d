"""Diagnostic: ulp error of the kernel tanh (cbn_param.hip tanh_fast) and of a
(13, 6) rational approximation against float64 tanh, in a float32 emulation
(fma as a float64 product + sum rounded once).  CPU only."""
import numpy as np
f32 = np.float32
def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)
def ulp_err(y, ref):
    ref32 = ref.astype(f32)
    sp = np.spacing(np.abs(ref32)).astype(np.float64)
    return np.abs(y.astype(np.float64) - ref) / sp
# sample: every float in [2^-20, 10] at stride, plus negatives
xs = np.linspace(0, 10, 4_000_001, dtype=np.float64).astype(f32)
xs = np.concatenate([xs, (np.logspace(-30, 0, 200000)).astype(f32)])
ref = np.tanh(xs.astype(np.float64))
# current
ax = np.abs(xs)
z = (ax * ax).astype(f32)
p = fma(z, f32(-5.70498872745e-3), np.full_like(z, 2.06390887954e-2))
p = fma(p, z, np.full_like(z, -5.37397155531e-2))
p = fma(p, z, np.full_like(z, 1.33314422036e-1))
p = fma(p, z, np.full_like(z, -3.33332819422e-1))
small = fma((p * z).astype(f32), ax, ax)
e = np.exp2((ax * f32(2.88539008177792681472)).astype(f32).astype(np.float64)).astype(f32)
u = (e + f32(1)).astype(f32)
r = (1.0 / u.astype(np.float64)).astype(f32)
big = fma(np.full_like(r, -2), r, np.full_like(r, 1))
cur = np.where(ax < 0.625, small, big)
err = ulp_err(cur, ref)
print("current: max ulp %.2f at x=%g, mean %.3f" % (err.max(), xs[err.argmax()], err.mean()))
# Eigen-style rational
A = [4.89352455891786e-03, 6.37261928875436e-04, 1.48572235717979e-05, 5.12229709037114e-08,
     -8.60467152213735e-11, 2.00018790482477e-13, -2.76076847742355e-16]
B = [4.89352518554385e-03, 2.26843463243900e-03, 1.18534705686654e-04, 1.19825839466702e-06]
for clampv in (7.90531110763549805, 9.0):
    x = np.clip(xs, -clampv, clampv).astype(f32)
    z = (x * x).astype(f32)
    p = np.full_like(z, A[6])
    for c in A[5::-1]:
        p = fma(p, z, np.full_like(z, c))
    p = (p * x).astype(f32)
    q = np.full_like(z, B[3])
    for c in B[2::-1]:
        q = fma(q, z, np.full_like(z, c))
    r = (1.0 / q.astype(np.float64)).astype(f32)
    qq = (p * r).astype(f32)
    res = fma(fma(-q, qq, p), r, qq)
    err = ulp_err(res, ref)
    print("rational clamp %.3f: max ulp %.2f at x=%g, mean %.3f; exact div max %.2f" % (
        clampv, err.max(), xs[err.argmax()], err.mean(),
        ulp_err((p.astype(np.float64) / q.astype(np.float64)).astype(f32), ref).max()))
    big = err > 2
    print("   frac > 2 ulp: %.5f; > 1 ulp: %.4f" % (big.mean(), (err > 1).mean()))

// Register-resident G1 formulas (force-inlined) for the latency-critical
// variable-base multiplication kernel.  Same formulas as curve.h (dbl-2009-l,
// add-2007-bl, madd-2007-bl) but inlined so the whole scalar multiplication
// lives in VGPRs with no call frames in scratch.
#pragma once
#include "curve.h"

namespace dx {

DX_HD void g1_dbl_i(G1J &p) {
  Fp A = fsqr(p.x), B = fsqr(p.y), C = fsqr(B);
  Fp D = fdbl(fsub(fsub(fsqr(fadd(p.x, B)), A), C));
  Fp E = fadd(fdbl(A), A);
  Fp F = fsqr(E);
  Fp X3 = fsub(F, fdbl(D));
  Fp C8 = fdbl(fdbl(fdbl(C)));
  Fp Y3 = fsub(fmul(E, fsub(D, X3)), C8);
  Fp Z3 = fdbl(fmul(p.y, p.z));
  p.x = X3;
  p.y = Y3;
  p.z = Z3;
}

// p += q (q affine, q != inf).  Handles p == inf and p == +-q.
DX_HD void g1_madd_i(G1J &p, const G1A &q) {
  if (p.is_inf()) {
    p = {q.x, q.y, Fp::one()};
    return;
  }
  Fp Z1Z1 = fsqr(p.z);
  Fp U2 = fmul(q.x, Z1Z1);
  Fp S2 = fmul(fmul(q.y, p.z), Z1Z1);
  Fp H = fsub(U2, p.x);
  Fp rr = fdbl(fsub(S2, p.y));
  if (H.is_zero()) {
    if (rr.is_zero()) {
      g1_dbl_i(p);
    } else {
      p = G1J::inf();
    }
    return;
  }
  Fp HH = fsqr(H);
  Fp I = fdbl(fdbl(HH));
  Fp J = fmul(H, I);
  Fp V = fmul(p.x, I);
  Fp X3 = fsub(fsub(fsqr(rr), J), fdbl(V));
  Fp Y3 = fsub(fmul(rr, fsub(V, X3)), fdbl(fmul(p.y, J)));
  Fp Z3 = fsub(fsub(fsqr(fadd(p.z, H)), Z1Z1), HH);
  p.x = X3;
  p.y = Y3;
  p.z = Z3;
}

// p += q, both Jacobian (q != inf).
DX_HD void g1_add_i(G1J &p, const G1J &q) {
  if (p.is_inf()) {
    p = q;
    return;
  }
  Fp Z1Z1 = fsqr(p.z), Z2Z2 = fsqr(q.z);
  Fp U1 = fmul(p.x, Z2Z2), U2 = fmul(q.x, Z1Z1);
  Fp S1 = fmul(fmul(p.y, q.z), Z2Z2), S2 = fmul(fmul(q.y, p.z), Z1Z1);
  Fp H = fsub(U2, U1);
  Fp rr = fdbl(fsub(S2, S1));
  if (H.is_zero()) {
    if (rr.is_zero()) {
      g1_dbl_i(p);
    } else {
      p = G1J::inf();
    }
    return;
  }
  Fp I = fsqr(fdbl(H));
  Fp J = fmul(H, I);
  Fp V = fmul(U1, I);
  Fp X3 = fsub(fsub(fsqr(rr), J), fdbl(V));
  Fp Y3 = fsub(fmul(rr, fsub(V, X3)), fdbl(fmul(S1, J)));
  Fp Z3 = fmul(fsub(fsub(fsqr(fadd(p.z, q.z)), Z1Z1), Z2Z2), H);
  p.x = X3;
  p.y = Y3;
  p.z = Z3;
}

}  // namespace dx

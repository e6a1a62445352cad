// secp256k1 group operations (y^2 = x^3 + 7, a = 0) on 10x26 field elements.
//
// Jacobian (X, Y, Z) represents (X/Z^2, Y/Z^3).  The formulas never use the
// curve constant b, so the same code runs unchanged on the isomorphic curves
// y^2 = x^3 + 7 C^6 that the variable-base table trick moves to (see
// scan_kernels.hip, build_odd_multiples).  None of the formulas handle the
// exceptional inputs (P == +-Q in an addition, the point at infinity); like the
// reference's gECC mixed add (src/cudasp_gpu.cu:58-59) they are only used where
// those cases have negligible probability for valid inputs.  The label step,
// where an exceptional input is reachable from user data, handles it
// explicitly (scan_kernels.hip, label_batch).
#pragma once
#include "secp256k1_fe.hpp"
#include "secp256k1_inv.hpp"

namespace cudasp {
CUDASP_HD void fe_inv(fe& r, const fe& a) { fe_inv_safegcd(r, a); }
}  // namespace cudasp

namespace cudasp {

struct ge {
  fe x, y;
};

struct gej {
  fe x, y, z;
};

// r = 2a  (dbl-2009-l, 2M + 5S).  r may alias a.
// Input magnitudes: x <= 7, y <= 17, z <= 8.  Output: x 1, y 17, z 2 -- the
// outputs of both dbl and madd are valid inputs of both, with one weak
// normalization each (mul/sqr take mag(a) * mag(b) <= 400).
CUDASP_HD void gej_double(gej& r, const gej& a) {
  fe A, B, C, D, E, t;
  FE_CHECK(a.x, 7, "dbl x");
  FE_CHECK(a.y, 17, "dbl y");
  FE_CHECK(a.z, 8, "dbl z");
  fe_sqr(A, a.x);          // A = X1^2                           (1)
  fe_sqr(B, a.y);          // B = Y1^2                           (1)
  fe_mul(r.z, a.y, a.z);   //                                    17 * 8
  fe_add(r.z, r.z, r.z);   // Z3 = 2 Y1 Z1                       (2)
  fe_sqr(C, B);            // C = B^2                            (1)
  fe_add(t, a.x, B);       // X1 + B                             (<= 8)
  fe_sqr(t, t);            //                                    (1)
  fe_sub<1>(t, t, A);      //                                    (3)
  fe_sub<1>(t, t, C);      //                                    (5)
  fe_add(D, t, t);         // D = 2((X1+B)^2 - A - C)            (10)
  fe_mul_int(E, A, 3);     // E = 3A                             (3)
  fe_sqr(t, E);            // F = E^2                            (1)
  fe_add(r.x, D, D);       //                                    (20)
  fe_sub<20>(r.x, t, r.x); // X3 = F - 2D                        (41)
  fe_normalize_weak(r.x);  //                                    (1)
  fe_sub<1>(t, D, r.x);    // D - X3                             (12)
  fe_mul(t, E, t);         //                                    3 * 12 -> (1)
  fe_mul_int(C, C, 8);     // 8C                                 (8)
  fe_sub<8>(r.y, t, C);    // Y3 = E (D - X3) - 8C               (17)
}

// Mixed addition r = a + b (b affine), 8M + 3S (madd-2004-hmv).  r may alias a.
// Input: a.x <= 7, a.y <= 17, a.z <= 8; b.x <= 2, b.y <= 17.
// Output: x 7, y 3, z 1.  If zr != nullptr it receives Z3 / Z1 (= H, mag 15).
CUDASP_HD void gej_add_ge(gej& r, const gej& a, const ge& b, fe* zr = nullptr) {
  fe z1z1, z1z1z1, u2, s2, h, rr, hh, hhh, v, t;
  FE_CHECK(a.x, 7, "add a.x");
  FE_CHECK(a.y, 17, "add a.y");
  FE_CHECK(a.z, 8, "add a.z");
  FE_CHECK(b.x, 2, "add b.x");
  FE_CHECK(b.y, 17, "add b.y");
  fe_sqr(z1z1, a.z);              // Z1^2                             (1)
  fe_mul(z1z1z1, z1z1, a.z);      // Z1^3                             (1)
  fe_mul(u2, b.x, z1z1);          // U2 = X2 Z1^2                     (1)
  fe_mul(s2, b.y, z1z1z1);        // S2 = Y2 Z1^3                     (1)
  fe_sub<7>(h, u2, a.x);          // H = U2 - X1                      (15)
  fe_sub<17>(rr, s2, a.y);        // R = S2 - Y1                      (35)
  fe_normalize_weak(rr);          //                                  (1)
  fe_mul(r.z, a.z, h);            // Z3 = Z1 H                        8 * 15 -> (1)
  if (zr) *zr = h;
  fe_sqr(hh, h);                  // HH                               15 * 15 -> (1)
  fe_mul(hhh, h, hh);             // HHH                              (1)
  fe_mul(v, a.x, hh);             // V = X1 HH                        (1)
  fe_mul(t, a.y, hhh);            // Y1 HHH                           (1)
  fe_sqr(r.x, rr);                // R^2                              (1)
  fe_sub<1>(r.x, r.x, hhh);       //                                  (3)
  fe_sub<1>(r.x, r.x, v);         //                                  (5)
  fe_sub<1>(r.x, r.x, v);         // X3 = R^2 - HHH - 2V              (7)
  fe_sub<7>(v, v, r.x);           // V - X3                           (15)
  fe_mul(v, rr, v);               //                                  (1)
  fe_sub<1>(r.y, v, t);           // Y3 = R (V - X3) - Y1 HHH         (3)
}

// Affine coordinates of a Jacobian point given 1/Z; fully normalized.
CUDASP_HD void gej_to_ge_zinv(ge& r, const gej& a, const fe& zinv) {
  fe zi2, zi3;
  fe_sqr(zi2, zinv);
  fe_mul(zi3, zi2, zinv);
  fe_mul(r.x, a.x, zi2);
  fe_mul(r.y, a.y, zi3);
  fe_normalize(r.x);
  fe_normalize(r.y);
}

CUDASP_HD void gej_set_ge(gej& r, const ge& a) {
  r.x = a.x;
  r.y = a.y;
  fe_set_int(r.z, 1);
}

// -a for a with y of magnitude <= 1; r.y has magnitude 2 (a valid gej_add_ge
// operand without normalization).
CUDASP_HD void ge_neg(ge& r, const ge& a) {
  r.x = a.x;
  fe_negate<1>(r.y, a.y);
}

}  // namespace cudasp

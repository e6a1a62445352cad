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

#if CUDASP_FE_LIMBS == 9
#include "secp256k1_group29.hpp"
#else
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

// Co-Z initial doubling with update (Meloni 2007, "DBLU"), 1M + 5S: for an
// affine T (normalized), d = 2T and t = T with the same Z = 2 T.y.
// Output: d.x 5, d.y 17, d.z 2; t.x 1, t.y 8, t.z 2.
CUDASP_HD void gej_dblu(gej& d, gej& t, const ge& T) {
  fe B, E, L, S, M, u;
  FE_CHECK(T.x, 1, "dblu x");
  FE_CHECK(T.y, 1, "dblu y");
  fe_sqr(B, T.x);          // B = X1^2                           (1)
  fe_sqr(E, T.y);          // E = Y1^2                           (1)
  fe_sqr(L, E);            // L = E^2                            (1)
  fe_add(u, T.x, E);       //                                    (2)
  fe_sqr(u, u);            //                                    (1)
  fe_sub<1>(u, u, B);      //                                    (3)
  fe_sub<1>(u, u, L);      //                                    (5)
  fe_add(S, u, u);         // S = 2((X1+E)^2 - B - L) = 4 X1 Y1^2 (10)
  fe_normalize_weak(S);    //                                    (1)
  fe_mul_int(M, B, 3);     // M = 3B                             (3)
  fe_sqr(d.x, M);          //                                    (1)
  fe_add(u, S, S);         //                                    (2)
  fe_sub<2>(d.x, d.x, u);  // X(2T) = M^2 - 2S                   (5)
  fe_sub<5>(u, S, d.x);    // S - X(2T)                          (11)
  fe_mul(d.y, M, u);       //                                    (1)
  fe_mul_int(L, L, 8);     // 8L = 8 Y1^4                        (8)
  fe_sub<8>(d.y, d.y, L);  // Y(2T) = M (S - X) - 8L             (17)
  fe_add(d.z, T.y, T.y);   // Z = 2 Y1                           (2)
  t.x = S;                 // T = (X1 (2Y1)^2, Y1 (2Y1)^3, 2Y1)
  t.y = L;
  t.z = d.z;
}

// Co-Z addition with update (Meloni 2007, "ZADDU"), 5M + 2S: p and q share Z;
// r = p + q and p becomes p with r's Z.  zr (if given) receives Z(r) / Z =
// X(p) - X(q) (mag 15).  Not for p == +-q.  r may not alias p or q.
// Input: p.x <= 5, p.y <= 17, p.z <= 2; q.x <= 5, q.y <= 8, q.z == p.z.
// Output: r.x 5, r.y 3, r.z 1; p.x 1, p.y 1, p.z 1.
CUDASP_HD void gej_zaddu(gej& r, gej& p, const gej& q, fe* zr = nullptr) {
  fe dx, dy, C, W1, W2, A1, t;
  FE_CHECK(p.x, 5, "zaddu p.x");
  FE_CHECK(p.y, 17, "zaddu p.y");
  FE_CHECK(p.z, 2, "zaddu p.z");
  FE_CHECK(q.x, 5, "zaddu q.x");
  FE_CHECK(q.y, 8, "zaddu q.y");
  fe_sub<5>(dx, p.x, q.x);     // X1 - X2                          (15)
  fe_sub<8>(dy, p.y, q.y);     // Y1 - Y2                          (33)
  fe_normalize_weak(dy);       //                                  (1)
  fe_sqr(C, dx);               // C = (X1 - X2)^2                  (1)
  fe_mul(W1, p.x, C);          // W1 = X1 C                        (1)
  fe_mul(W2, q.x, C);          // W2 = X2 C                        (1)
  fe_sub<1>(t, W1, W2);        //                                  (3)
  fe_mul(A1, p.y, t);          // A1 = Y1 (W1 - W2)                17 * 3 -> (1)
  fe_sqr(r.x, dy);             // D = (Y1 - Y2)^2                  (1)
  fe_sub<1>(r.x, r.x, W1);     //                                  (3)
  fe_sub<1>(r.x, r.x, W2);     // X3 = D - W1 - W2                 (5)
  fe_sub<5>(t, W1, r.x);       // W1 - X3                          (11)
  fe_mul(r.y, dy, t);          //                                  (1)
  fe_sub<1>(r.y, r.y, A1);     // Y3 = (Y1 - Y2)(W1 - X3) - A1     (3)
  fe_mul(r.z, p.z, dx);        // Z3 = Z (X1 - X2)                 2 * 15 -> (1)
  if (zr) *zr = dx;
  p.x = W1;
  p.y = A1;
  p.z = r.z;
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
#endif

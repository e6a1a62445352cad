// secp256k1 group operations for the 9 x 29-bit field layout
// (CUDASP_FE_LIMBS=9; included by secp256k1_group.hpp instead of the 10 x 26
// formulas).  Same functions and meaning; the formulas are chosen and the
// weak normalizations placed for the tight magnitude budget of
// secp256k1_fe29.hpp (mul: mag(a) * mag(b) <= 7, sqr: <= 2, sums <= 7).
//
// Point contract shared by the main-loop operations: a Jacobian point fed to
// gej_double / gej_add_ge has x <= 1, y <= 2, z <= 2 (y = 2: a point set from a
// negated affine entry, or a doubling's output); gej_add_ge returns
// (1, 1, 1), gej_double (1, 2, 1).  Affine operands: x <= 1, y <= 2 (a
// normalized y, or its negation).
#pragma once

namespace cudasp {

struct ge {
  fe x, y;
};

struct gej {
  fe x, y, z;
};

// r = 2a (3M + 4S, the halved form: Z3 = Y1 Z1, L = 3/2 X1^2,
// X3 = L^2 - 2 X1 Y1^2, Y3 = -(L (X3 - X1 Y1^2) + Y1^4)).  X3 and Y3 each come
// out of one fused reduction (fe_sqr_add, fe_mulsqr).  r may alias a.
// Output: x = z = 1, y = 2.
CUDASP_HD void gej_double(gej& r, const gej& a) {
  fe S, L, T, U;
  FE_CHECK(a.x, 1, "dbl x");
  FE_CHECK(a.y, 2, "dbl y");
  FE_CHECK(a.z, 2, "dbl z");
  fe_mul(r.z, a.z, a.y);   // Z3 = Y1 Z1                         2 * 2 -> (1)
  fe_sqr(S, a.y);          // S = Y1^2                           (1)
  fe_sqr3(L, a.x);         // 3 X1^2                             (1)
  fe_half(L, L);           // L = 3/2 X1^2                       (2)
  fe_mul(T, S, a.x);       //                                    (1)
  fe_negate<1>(T, T);      // T = -X1 S                          (2)
  fe_add(U, T, T);         // 2T                                 (4)
  fe_sqr_add(r.x, L, U);   // X3 = L^2 + 2T                      (1)
  fe_add(U, r.x, T);       // X3 + T                             (3)
  fe_mulsqr(r.y, L, U, S); // L (X3 + T) + S^2                   2 * 3 + 1 -> (1)
  fe_negate<1>(r.y, r.y);  // Y3                                 (2)
}

// Mixed addition r = a + b (b affine), 8M + 3S (madd-2004-hmv).  r may alias a.
// If zr != nullptr it receives Z3 / Z1 (= H, mag 1).  H, R and X3 each take
// their subtrahends inside the product's reduction (fe_mul_add, fe_sqr_add)
// and Y3 = R (V - X3) + (-Y1) HHH is one fused reduction (fe_mul2).
CUDASP_HD void gej_add_ge(gej& r, const gej& a, const ge& b, fe* zr = nullptr) {
  fe z1z1, z1z1z1, u2, h, rr, hh, hhh, v, ny, w;
  FE_CHECK(a.x, 1, "add a.x");
  FE_CHECK(a.y, 2, "add a.y");
  FE_CHECK(a.z, 2, "add a.z");
  FE_CHECK(b.x, 1, "add b.x");
  FE_CHECK(b.y, 2, "add b.y");
  fe_sqr(z1z1, a.z);               // Z1^2                            (1)
  fe_mul(z1z1z1, z1z1, a.z);       // Z1^3                            (1)
  fe_negate<1>(u2, a.x);           // -X1                             (2)
  fe_mul_add(h, b.x, z1z1, u2);    // H = X2 Z1^2 - X1                (1)
  fe_negate<2>(ny, a.y);           // -Y1                             (3)
  fe_mul_add(rr, b.y, z1z1z1, ny); // R = Y2 Z1^3 - Y1                2 * 1 -> (1)
  fe_mul(r.z, a.z, h);             // Z3 = Z1 H                       (1)
  if (zr) *zr = h;
  fe_sqr(hh, h);                   // HH                              (1)
  fe_mul(hhh, h, hh);              // HHH                             (1)
  fe_mul(v, a.x, hh);              // V = X1 HH                       (1)
  fe_add(w, v, v);
  fe_add_to(w, hhh);               // HHH + 2V                        (3)
  fe_negate<3>(w, w);              //                                 (4)
  fe_sqr_add(r.x, rr, w);          // X3 = R^2 - HHH - 2V             (1)
  fe_sub<1>(v, v, r.x);            // V - X3                          (3)
  fe_mul2(r.y, rr, v, ny, hhh);    // Y3 = R (V - X3) - Y1 HHH        1 * 3 + 3 * 1 -> (1)
}

// ---- Stage-A ladder forms: Y kept doubled ("Yh" = 2Y), sign tracked outside.
// The doubling then needs no halving (M = 3 X^2 instead of 3/2 X^2) and no
// final negation: it returns -2Q.  The mixed addition halves R once instead.
// A stored triple (X, Yh, Z) stands for the Jacobian point Q = (X, Yh / 2, Z).

// r = -2a (Yh form).  Input: x <= 1, yh <= 2, z <= 2.  Output: (1, 1, 1).
// Z3 = Yh Z (= 2 Y Z), A = Yh^2 (= 4 Y^2), B = X A (= 4 X Y^2), M = 3 X^2,
// X3 = M^2 - 2 B, Yh3 = 2 M (X3 - B) + A^2 (= -2 Y3).  r may alias a.
CUDASP_HD void gej_double_neg_yh(gej& r, const gej& a) {
  fe A, M, B, nb, w;
  FE_CHECK(a.x, 1, "dblh x");
  FE_CHECK(a.y, 2, "dblh y");
  FE_CHECK(a.z, 2, "dblh z");
  fe_mul(r.z, a.z, a.y);    // Z3 = Yh Z                          (1)
  fe_sqr(A, a.y);           // A = Yh^2                           (1)
  fe_sqr3(M, a.x);          // M = 3 X^2                          (1)
  fe_mul(B, a.x, A);        // B = X A                            (1)
  fe_negate<1>(nb, B);      // -B                                 (2)
  fe_add(w, nb, nb);        // -2B                                (4)
  fe_sqr_add(r.x, M, w);    // X3 = M^2 - 2B                      (1)
  fe_add_x2(w, r.x, nb);    // 2 (X3 - B)                         (6)
  fe_mulsqr(r.y, M, w, A);  // Yh3' = M 2 (X3 - B) + A^2          1 * 6 + 1 -> (1)
}

// r = a + b (Yh form, b affine with yh = 2y, possibly negated).  Input:
// a = (1, 1, 2), b = (1, 3).  Output (1, 1, 1).  H = X2 Z1^2 - X1,
// R' = Yh2 Z1^3 - Yh1 (= 2R), R = R' / 2, X3 = R^2 - HHH - 2V,
// Yh3 = R' (V - X3) - Yh1 HHH, Z3 = Z1 H.  r may alias a.
CUDASP_HD void gej_add_ge_yh(gej& r, const gej& a, const ge& b) {
  fe z1z1, z1z1z1, t, h, rr, r1, hh, hhh, v, ny, w;
  FE_CHECK(a.x, 1, "addh a.x");
  FE_CHECK(a.y, 1, "addh a.y");
  FE_CHECK(a.z, 2, "addh a.z");
  FE_CHECK(b.x, 1, "addh b.x");
  FE_CHECK(b.y, 3, "addh b.y");
  fe_sqr(z1z1, a.z);               // Z1^2                            (1)
  fe_mul(z1z1z1, z1z1, a.z);       // Z1^3                            (1)
  fe_negate<1>(t, a.x);            // -X1                             (2)
  fe_mul_add(h, b.x, z1z1, t);     // H = X2 Z1^2 - X1                (1)
  fe_negate<1>(ny, a.y);           // -Yh1                            (2)
  fe_mul_add(rr, b.y, z1z1z1, ny); // R' = Yh2 Z1^3 - Yh1             3 * 1 -> (1)
  fe_half(r1, rr);                 // R                               (2)
  fe_mul(r.z, a.z, h);             // Z3 = Z1 H                       (1)
  fe_sqr(hh, h);                   // HH                              (1)
  fe_mul(hhh, h, hh);              // HHH                             (1)
  fe_mul(v, a.x, hh);              // V = X1 HH                       (1)
  fe_add(w, v, v);
  fe_add_to(w, hhh);               // HHH + 2V                        (3)
  fe_negate<3>(w, w);              //                                 (4)
  fe_sqr_add(r.x, r1, w);          // X3 = R^2 - HHH - 2V             (1)
  fe_sub<1>(v, v, r.x);            // V - X3                          (3)
  fe_mul2(r.y, rr, v, ny, hhh);    // Yh3 = R' (V - X3) - Yh1 HHH     1 * 3 + 2 * 1 -> (1)
}

// Co-Z initial doubling with update: for an affine, normalized T, d = 2T and
// t = T with the same Z = T.y.  The halved doubling already forms
// X1 Y1^2 and Y1^4, which are T's coordinates at Z = Y1.
// Output: d = (1, 1, 1), t = (1, 1, 1).
CUDASP_HD void gej_dblu(gej& d, gej& t, const ge& T) {
  fe S, L, XS, U;
  FE_CHECK(T.x, 1, "dblu x");
  FE_CHECK(T.y, 1, "dblu y");
  fe_sqr(S, T.y);           // S = Y1^2                          (1)
  fe_sqr(L, T.x);
  fe_mul_int(L, L, 3);
  fe_half(L, L);            // L = 3/2 X1^2                      (2.5)
  fe_normalize_weak(L);     //                                   (1)
  fe_mul(XS, T.x, S);       // X1 S                              (1)
  fe_sqr(d.x, L);
  fe_sub<1>(d.x, d.x, XS);  //                                   (3)
  fe_sub<1>(d.x, d.x, XS);  // X(2T) = L^2 - 2 X1 S              (5)
  fe_normalize_weak(d.x);   //                                   (1)
  fe_sub<1>(U, d.x, XS);    // X3 - X1 S                         (3)
  fe_mul(d.y, L, U);        //                                   (1)
  fe_sqr(S, S);             // Y1^4                              (1)
  fe_add_to(d.y, S);        //                                   (2)
  fe_negate<2>(d.y, d.y);   // Y(2T) = -(L (X3 - X1 S) + Y1^4)   (3)
  fe_normalize_weak(d.y);   //                                   (1)
  d.z = T.y;                // Z = Y1
  t.x = XS;                 // T = (X1 Y1^2, Y1^4, Y1)
  t.y = S;
  t.z = T.y;
}

// Co-Z addition with update (Meloni 2007, "ZADDU"), 5M + 2S: p and q share Z;
// r = p + q and p becomes p with r's Z.  zr (if given) receives Z(r) / Z =
// X(p) - X(q) (mag 1).  Not for p == +-q.  r may not alias p or q.
// Input: p = (1, 1, 1), q = (1, 3, 1).  Output: r = (1, 3, 1), p = (1, 1, 1).
CUDASP_HD void gej_zaddu(gej& r, gej& p, const gej& q, fe* zr = nullptr) {
  fe dx, dy, C, W1, W2, A1, t;
  FE_CHECK(p.x, 1, "zaddu p.x");
  FE_CHECK(p.y, 1, "zaddu p.y");
  FE_CHECK(q.x, 1, "zaddu q.x");
  FE_CHECK(q.y, 3, "zaddu q.y");
  fe_sub<1>(dx, p.x, q.x);     // X1 - X2                          (3)
  fe_normalize_weak(dx);       //                                  (1)
  fe_sub<3>(dy, p.y, q.y);     // Y1 - Y2                          (5)
  fe_normalize_weak(dy);       //                                  (1)
  fe_sqr(C, dx);               // C = (X1 - X2)^2                  (1)
  fe_mul(W1, p.x, C);          // W1 = X1 C                        (1)
  fe_mul(W2, q.x, C);          // W2 = X2 C                        (1)
  fe_sub<1>(t, W1, W2);        //                                  (3)
  fe_mul(A1, p.y, t);          // A1 = Y1 (W1 - W2)                (1)
  fe_sqr(r.x, dy);             // D = (Y1 - Y2)^2                  (1)
  fe_sub<1>(r.x, r.x, W1);     //                                  (3)
  fe_sub<1>(r.x, r.x, W2);     // X3 = D - W1 - W2                 (5)
  fe_normalize_weak(r.x);      //                                  (1)
  fe_sub<1>(t, W1, r.x);       // W1 - X3                          (3)
  fe_mul(r.y, dy, t);          //                                  (1)
  fe_sub<1>(r.y, r.y, A1);     // Y3 = (Y1 - Y2)(W1 - X3) - A1     (3)
  fe_mul(r.z, p.z, dx);        // Z3 = Z (X1 - X2)                 (1)
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

// -a for a with y of magnitude <= 1; r.y has magnitude 2.
CUDASP_HD void ge_neg(ge& r, const ge& a) {
  r.x = a.x;
  fe_negate<1>(r.y, a.y);
}

}  // namespace cudasp

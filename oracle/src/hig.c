/*
 * hig.c -- hypergeometric-inverse-gamma numerics of code/hyperg.cpp (TEST INFRASTRUCTURE ONLY).
 * Each function restates the reference function named in its comment; the error
 * paths reproduce the reference's GSL status mapping (hg:30-45).
 */
#include "oracle.h"
#include <math.h>

#define GSL_SUCCESS  0
#define GSL_EMAXITER 11

/* HDPM_OPT_HIG_LOGSPACE mirror (extension, not the reference): norm_const2 and lF_conK2
 * take log 2F1 from orc_log_hyperg_2F1. */
static int g_hig_logspace = 0;
void orc_set_hig_logspace(int on) { g_hig_logspace = on != 0; }

/* hg:11-48 norm_const2(d, c, m).  *err = ORC_E_GSL where the reference throws. */
double orc_norm_const2(double d, double c, double m, int* err) {
    double z = (m - 1) / m;
    if (g_hig_logspace) {
        double lv;
        int st = orc_log_hyperg_2F1(d + c, 1, d + 2, z, &lv);
        if (st != GSL_SUCCESS) {
            if (st == GSL_EMAXITER) return -INFINITY;
            if (err) *err = ORC_E_GSL;
            return NAN;
        }
        if (!isfinite(lv)) {
            if (err) *err = ORC_E_GSL;
            return NAN;
        }
        return log(d + 1) + (d + c) * log(m) - lv;
    }
    double alpha = d + c;
    double beta = 1;
    double gamma = d + 2;
    double val;
    int stat = orc_hyperg_2F1(alpha, beta, gamma, z, &val);
    if (stat != GSL_SUCCESS) {
        if (stat == GSL_EMAXITER) return -INFINITY;
        /* GSL_EOVRFLW is never raised by the series branch (it overflows to +inf and
         * returns success, caught below); every other status throws. */
        if (err) *err = ORC_E_GSL;
        return NAN;
    }
    if (!isfinite(val) || val == 0) {
        if (err) *err = ORC_E_GSL;
        return NAN;
    }
    return log(d + 1) + (d + c) * log(m) - log(val);
}

/* hg:51-78 hyperg2: 2F1 or NaN on any GSL failure. */
double orc_hyperg2(double a, double b, double c, double x) {
    double val;
    int stat = orc_hyperg_2F1(a, b, c, x, &val);
    if (stat != GSL_SUCCESS) return NAN;
    return val;
}

/* hg:183-217 lF_conK2 */
double orc_lF_conK2(double u, double d, double c, double m, double lK) {
    if (u == 0) return -INFINITY;
    if (u == 1) return 0;
    double x = u * (m - 1) / (1 + u * (m - 1));
    double lapp;
    if (g_hig_logspace) {
        if (orc_log_hyperg_2F1(1, d + c, d + 2, x, &lapp) != GSL_SUCCESS) lapp = NAN;
    } else {
        lapp = log(orc_hyperg2(1, d + c, d + 2, x));
    }
    double out = lK - log(d + 1) + (d + 1) * log(u) - (d + c) * log(1 + u * (m - 1)) + lapp;
    return out;
}

/* hg:221-287 bisec_hyper2 */
double orc_bisec_hyper2(double d, double c, double m, double Omega, int* err) {
    double centro = 0.5;
    int e = ORC_OK;
    double lK = orc_norm_const2(d, c, m, &e);
    if (e) { if (err) *err = e; return NAN; }
    double app = orc_lF_conK2(centro, d, c, m, lK) - log(Omega);
    double su, giu;
    int counter = 1;
    int max_count = 150;
    if (app < 0) { giu = 0.5; su = 1; }
    else { giu = 0; su = 0.5; }
    while (((su - giu) > 0.000000001) & (counter < max_count)) {
        centro = (su + giu) / 2;
        app = orc_lF_conK2(centro, d, c, m, lK) - log(Omega);
        if (app < 0) giu = centro;
        else su = centro;
        counter = counter + 1;
    }
    return centro;
}

/* hg:346-378 rhig with n = 1.  The `(m-1)/m > 4/5` clause is integer 4/5 == 0. */
double orc_rhig1(orc_rng* r, double v, double w, double m, int* err) {
    double out;
    if (orc_qbeta01_lt(w + 1, v - 1, (m - 1) / m) && (m - 1) / m > 4 / 5) {
        double x = orc_rbeta(r, w + 1, v - 1);
        while (x > (m - 1) / m) x = orc_rbeta(r, w + 1, v - 1);
        out = x / ((m - 1) * (1 - x));
    } else {
        double Omega = orc_unif_rand(r);   /* R::runif(0, 1) */
        int e = ORC_OK;
        out = orc_bisec_hyper2(w, v, m, Omega, &e);
        if (e) { if (err) *err = e; return NAN; }
    }
    return -1 / log(out);
}

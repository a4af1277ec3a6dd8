/* ORACLE (test infrastructure only): small dense fp64 kernels, row-major. */
#include <math.h>
#include "oracle.h"

int orc_chol(int n, double *A)
{
    for (int j = 0; j < n; j++) {
        double d = A[j * n + j];
        for (int k = 0; k < j; k++) d -= A[j * n + k] * A[j * n + k];
        if (!(d > 0.0)) return -1;
        d = sqrt(d);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[i * n + j];
            for (int k = 0; k < j; k++) s -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = s / d;
        }
        for (int i = 0; i < j; i++) A[i * n + j] = 0.0;
    }
    return 0;
}

void orc_chol_solve(int n, const double *L, double *x)
{
    for (int i = 0; i < n; i++) {
        double s = x[i];
        for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
        x[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = x[i];
        for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
        x[i] = s / L[i * n + i];
    }
}

int orc_lu(int n, double *A, int *piv)
{
    int ok = 0;
    for (int k = 0; k < n; k++) {
        int p = k; double mx = fabs(A[k * n + k]);
        for (int i = k + 1; i < n; i++) if (fabs(A[i * n + k]) > mx) { mx = fabs(A[i * n + k]); p = i; }
        piv[k] = p;
        if (mx == 0.0) { ok = -1; continue; }
        if (p != k) for (int j = 0; j < n; j++) { double t = A[k * n + j]; A[k * n + j] = A[p * n + j]; A[p * n + j] = t; }
        double inv = 1.0 / A[k * n + k];
        for (int i = k + 1; i < n; i++) {
            double l = A[i * n + k] * inv;
            A[i * n + k] = l;
            if (l != 0.0) for (int j = k + 1; j < n; j++) A[i * n + j] -= l * A[k * n + j];
        }
    }
    return ok;
}

void orc_lu_solve(int n, const double *LU, const int *piv, double *x)
{
    for (int k = 0; k < n; k++) { int p = piv[k]; if (p != k) { double t = x[k]; x[k] = x[p]; x[p] = t; } }
    for (int i = 0; i < n; i++) { double s = x[i]; for (int k = 0; k < i; k++) s -= LU[i * n + k] * x[k]; x[i] = s; }
    for (int i = n - 1; i >= 0; i--) { double s = x[i]; for (int k = i + 1; k < n; k++) s -= LU[i * n + k] * x[k]; x[i] = s / LU[i * n + i]; }
}

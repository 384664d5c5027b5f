/*
 * oracle/solver_impl.h — TEST INFRASTRUCTURE ONLY (see oracle/README.md).
 *
 * Generic restatement of the reference's GN / LM solver loop over a family's
 * per-unknown functions, instantiated for REAL = float and REAL = double by
 * oracle/solver.c. Follows API/src/solverGPUGaussNewton.t:
 *   init (:1766-1897): prevCost = cost
 *   step (:1913-2349): PCGInit1 (:521-563) [+ LM: PCGSaveSSq, PCGComputeCtC,
 *   PCGFinalizeDiagonal :1042-1103], lIterations x {PCGStep1, PCGStep2 or the
 *   residual-reset halves :738-801, PCGStep3, alpha_num = beta_num, LM zeta exit
 *   :2211-2220}, LM model cost, savePreviousUnknowns, PCGLinearUpdate, cost, LM
 *   accept / reject with the trust-region update (:2247-2292).
 * Scalar sums are accumulated in OACC (double for REAL = float, long double for REAL =
 * double: the fp64 truth, see oracle/iw_impl.h); opt_float arithmetic elsewhere.
 */
#ifndef REAL
#error define REAL
#endif

#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

static REAL CAT(ginv_, REAL)(REAL d) { REAL s = (REAL)1 + (REAL)sqrt((double)d); return (REAL)1 / (s * s); }

/* Returns the number of steps that returned 1; costs[0] = initial cost, costs[i] after
 * step i (the reference's Opt_ProblemCurrentCost after each Step). */
static int CAT(oracle_solve_, REAL)(CAT(oracle_problem_, REAL)* P, int lm, const oracle_params* sp,
                                    double* costs) {
    const long long n = P->n;
    REAL *r = calloc(n, sizeof(REAL)), *diag = calloc(n, sizeof(REAL)), *pre = calloc(n, sizeof(REAL));
    REAL *p = calloc(n, sizeof(REAL)), *Ap = calloc(n, sizeof(REAL)), *d = calloc(n, sizeof(REAL));
    REAL *b = calloc(n, sizeof(REAL)), *CtC = calloc(n, sizeof(REAL)), *SSq = calloc(n, sizeof(REAL));
    REAL *Ad = calloc(n, sizeof(REAL)), *CtCp = calloc(n, sizeof(REAL));
    double prev_cost = P->cost(P->ctx);
    float radius = sp->trust_region_radius, decrease = sp->radius_decrease_factor;
    costs[0] = prev_cost;
    int done = 0, completed = 0;
    for (int it = 0; it < sp->nIterations; ++it) {
        /* PCGInit1 */
        P->jtf(P->ctx, r, diag);
        OACC alpha_num = 0.0;
        for (long long e = 0; e < n; ++e) {
            d[e] = 0;
            REAL w = P->act[e] ? CAT(ginv_, REAL)(P->use_pre ? diag[e] : (REAL)1) : (REAL)0;
            pre[e] = w;
            p[e] = w * r[e];
            alpha_num += (double)r[e] * p[e];
        }
        REAL Q0 = 0;
        if (lm) {
            if (it == 0) for (long long e = 0; e < n; ++e) SSq[e] = pre[e];
            const REAL rad = (REAL)radius, inv_rad = (REAL)1 / rad;
            alpha_num = 0.0;
            for (long long e = 0; e < n; ++e) {
                if (!P->act[e]) { CtC[e] = pre[e] = b[e] = p[e] = 0; continue; }
                const REAL unc = diag[e] * inv_rad;
                const REAL cm = ((REAL)1 / SSq[e]) / rad;
                REAL lo = (REAL)sp->min_lm_diagonal * cm, hi = (REAL)sp->max_lm_diagonal * cm;
                REAL c = unc < lo ? lo : unc;
                if (c > hi) c = hi;
                CtC[e] = c;
                pre[e] = (REAL)1 / (c + rad * unc);
                b[e] = r[e];
                p[e] = pre[e] * r[e];
                alpha_num += (double)r[e] * p[e];
            }
        }
        if (P->materialize) P->materialize(P->ctx);
        for (int li = 0; li < sp->lIterations; ++li) {
            /* PCGStep1 (+ CtC p for LM), or the materialized SpMV + PCGStep1_Finish */
            OACC alpha_den = P->apply_mat ? P->apply_mat(P->ctx, p, Ap) : P->apply(P->ctx, p, Ap);
            if (lm && !P->apply_mat) {
                for (long long e = 0; e < n; ++e) {
                    Ap[e] += CtC[e] * p[e];
                    alpha_den += (double)p[e] * (CtC[e] * p[e]);
                }
            }
            const REAL alpha = (REAL)(alpha_num / alpha_den);
            OACC beta_num = 0.0, q = 0.0;
            const int reset = lm && ((li + 1) % (sp->residual_reset_period > 0 ? sp->residual_reset_period : 1)) == 0;
            if (reset) {
                for (long long e = 0; e < n; ++e) d[e] = d[e] + alpha * p[e];
                P->apply(P->ctx, d, Ad);
                for (long long e = 0; e < n; ++e) {
                    Ad[e] += CtC[e] * d[e];
                    r[e] = b[e] - Ad[e];
                    const REAL z = P->use_pre ? pre[e] * r[e] : r[e];
                    beta_num += (double)z * r[e];
                    q += (double)((REAL)0.5 * (d[e] * (r[e] + b[e])));
                }
            } else {
                for (long long e = 0; e < n; ++e) {
                    d[e] = d[e] + alpha * p[e];
                    r[e] = r[e] - alpha * Ap[e];
                    const REAL z = P->use_pre ? pre[e] * r[e] : r[e];
                    beta_num += (double)z * r[e];
                    if (lm) q += (double)((REAL)0.5 * (d[e] * (r[e] + b[e])));
                }
            }
            const REAL beta = (REAL)(beta_num / alpha_num);
            for (long long e = 0; e < n; ++e) {
                const REAL z = P->use_pre ? pre[e] * r[e] : r[e];
                p[e] = z + beta * p[e];
            }
            alpha_num = beta_num;
            if (lm) {
                const REAL Q1 = (REAL)q;
                const REAL zeta = (REAL)(li + 1) * (Q1 - Q0) / Q1;
                if (zeta < (REAL)sp->q_tolerance) break;
                Q0 = Q1;
            }
        }
        if (!lm) {
            if (sp->lIterations > 0) P->update(P->ctx, d);
            prev_cost = P->cost(P->ctx);
            costs[it + 1] = prev_cost;
            ++completed;
            continue;
        }
        const REAL model_cost = (REAL)P->model_cost(P->ctx, d);
        if (sp->lIterations > 0) { P->save(P->ctx); P->update(P->ctx, d); }
        const REAL new_cost = (REAL)P->cost(P->ctx);
        const REAL prevc = (REAL)prev_cost;
        const REAL model_change = prevc - model_cost, cost_change = prevc - new_cost;
        const REAL rel = cost_change / model_change;
        if (getenv("ORACLE_DEBUG")) fprintf(stderr, "it %d prev %g model %g new %g rel %g radius %g\n", it, (double)prevc, (double)model_cost, (double)new_cost, (double)rel, radius);
        if (cost_change >= 0 && rel > (REAL)sp->min_relative_decrease) {
            if (cost_change <= prevc * (REAL)sp->function_tolerance) { done = 1; break; }
            const REAL qq = rel;
            const REAL mf = (REAL)(1.0 / 3.0);
            const REAL tmp = (REAL)1 - (REAL)pow((double)((REAL)2 * qq - (REAL)1), 3.0);
            float rr = (float)((REAL)radius / (mf > tmp ? mf : tmp));
            radius = rr < sp->max_trust_region_radius ? rr : sp->max_trust_region_radius;
            decrease = 2.0f;
            prev_cost = (double)new_cost;
        } else {
            if (sp->lIterations > 0) P->revert(P->ctx);
            radius = radius / decrease;
            decrease = 2.0f * decrease;
            if (radius <= sp->min_trust_region_radius) { done = 1; break; }
        }
        costs[it + 1] = prev_cost;
        ++completed;
    }
    free(r); free(diag); free(pre); free(p); free(Ap); free(d); free(b); free(CtC); free(SSq); free(Ad); free(CtCp);
    (void)done;
    return completed;
}

#undef CAT
#undef CAT2

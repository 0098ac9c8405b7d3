/* ORACLE (test infrastructure only) — basis factorization driver.
 * Restates glpbfd.js (GLPK 4.49): bfd_create_it :10, bfd_set_parm :31,
 * bfd_factorize :47, bfd_ftran :148, bfd_btran :159, bfd_update_it :170,
 * bfd_get_count :225. */
#include "orc.h"

orc_bfd *bfd_create_it(void)
{
    orc_bfd *bfd = (orc_bfd *)orc_alloc(1, sizeof(orc_bfd));
    bfd->type = GLP_BF_FT;
    bfd->lu_size = 0;
    bfd->piv_tol = 0.10;
    bfd->piv_lim = 4;
    bfd->suhl = 1;
    bfd->eps_tol = 1e-15;
    bfd->max_gro = 1e+10;
    bfd->nfs_max = 100;
    bfd->upd_tol = 1e-6;
    bfd->nrs_max = 100;
    bfd->rs_size = 1000;
    bfd->upd_lim = -1;
    bfd->upd_cnt = 0;
    return bfd;
}

void bfd_delete_it(orc_bfd *bfd)
{
    if (!bfd) return;
    fhv_delete_it(bfd->fhv);
    lpf_delete_it(bfd->lpf);
    orc_free(bfd);
}

void bfd_set_parm(orc_bfd *bfd, const orc_bfcp *parm)
{
    ORC_ASSERT(bfd != NULL);
    bfd->type = parm->type;
    bfd->lu_size = parm->lu_size;
    bfd->piv_tol = parm->piv_tol;
    bfd->piv_lim = parm->piv_lim;
    bfd->suhl = parm->suhl;
    bfd->eps_tol = parm->eps_tol;
    bfd->max_gro = parm->max_gro;
    bfd->nfs_max = parm->nfs_max;
    bfd->upd_tol = parm->upd_tol;
    bfd->nrs_max = parm->nrs_max;
    bfd->rs_size = parm->rs_size;
}

int bfd_factorize(orc_bfd *bfd, int m, const int *bh, orc_col_fn col, void *info)
{
    orc_luf *luf;
    int nov = 0, ret;
    ORC_ASSERT(bfd != NULL);
    ORC_ASSERT(1 <= m);
    bfd->valid = 0;
    switch (bfd->type) {
    case GLP_BF_FT:
        lpf_delete_it(bfd->lpf); bfd->lpf = NULL;
        if (bfd->fhv == NULL) { bfd->fhv = fhv_create_it(); nov = 1; }
        break;
    case GLP_BF_BG:
    case GLP_BF_GR:
        fhv_delete_it(bfd->fhv); bfd->fhv = NULL;
        if (bfd->lpf == NULL) { bfd->lpf = lpf_create_it(); nov = 1; }
        break;
    default:
        ORC_ASSERT(0);
    }
    luf = bfd->fhv ? bfd->fhv->luf : bfd->lpf->luf;
    if (nov) luf->new_sva = bfd->lu_size;
    luf->piv_tol = bfd->piv_tol;
    luf->piv_lim = bfd->piv_lim;
    luf->suhl = bfd->suhl;
    luf->eps_tol = bfd->eps_tol;
    luf->max_gro = bfd->max_gro;
    if (bfd->fhv != NULL) {
        if (nov) bfd->fhv->hh_max = bfd->nfs_max;
        bfd->fhv->upd_tol = bfd->upd_tol;
    }
    if (bfd->lpf != NULL) {
        if (nov) bfd->lpf->n_max = bfd->nrs_max;
        if (nov) bfd->lpf->v_size = bfd->rs_size;
    }
    if (bfd->fhv != NULL) {
        ret = fhv_factorize(bfd->fhv, m, col, info);
        if (ret == 1) return BFD_ESING;
        if (ret == 2) return BFD_ECOND;
        ORC_ASSERT(ret == 0);
    } else {
        ret = lpf_factorize(bfd->lpf, m, bh, col, info);
        if (ret == LPF_ESING) return BFD_ESING;
        if (ret == LPF_ECOND) return BFD_ECOND;
        ORC_ASSERT(ret == 0);
        bfd->lpf->scf->t_opt = (bfd->type == GLP_BF_BG ? SCF_TBG : SCF_TGR);
    }
    bfd->valid = 1;
    bfd->upd_cnt = 0;
    return 0;
}

void bfd_ftran(orc_bfd *bfd, double *x)
{
    ORC_ASSERT(bfd != NULL);
    ORC_ASSERT(bfd->valid);
    if (bfd->fhv != NULL) fhv_ftran(bfd->fhv, x);
    else lpf_ftran(bfd->lpf, x);
}

void bfd_btran(orc_bfd *bfd, double *x)
{
    ORC_ASSERT(bfd != NULL);
    ORC_ASSERT(bfd->valid);
    if (bfd->fhv != NULL) fhv_btran(bfd->fhv, x);
    else lpf_btran(bfd->lpf, x);
}

int bfd_update_it(orc_bfd *bfd, int j, int bh, int len, const int *ind, int idx, const double *val)
{
    int ret;
    ORC_ASSERT(bfd != NULL);
    ORC_ASSERT(bfd->valid);
    if (bfd->fhv != NULL) {
        ret = fhv_update_it(bfd->fhv, j, len, ind, idx, val);
        switch (ret) {
        case 0: break;
        case 1: bfd->valid = 0; return BFD_ESING;
        case 3: bfd->valid = 0; return BFD_ECHECK;
        case 4: bfd->valid = 0; return BFD_ELIMIT;
        case 5: bfd->valid = 0; return BFD_EROOM;
        default: ORC_ASSERT(0);
        }
    } else {
        ret = lpf_update_it(bfd->lpf, j, bh, len, ind, idx, val);
        switch (ret) {
        case 0: break;
        case LPF_ESING: bfd->valid = 0; return BFD_ESING;
        case LPF_ELIMIT: bfd->valid = 0; return BFD_ELIMIT;
        default: ORC_ASSERT(0);
        }
    }
    bfd->upd_cnt++;
    return 0;
}

int bfd_get_count(orc_bfd *bfd)
{
    ORC_ASSERT(bfd != NULL);
    ORC_ASSERT(bfd->valid);
    return bfd->upd_cnt;
}

/*
 * conv_detect.c -- decentralised global convergence detection of the
 * asynchronous multisplitting drivers: Algorithm 5.15 ("practical version of
 * convergence detection", Bahi, Contassot-Vivier, Couturier, Parallel
 * Iterative Algorithms) as the reference implements it in
 * src/utils/conv_detection_prime.c, over the amsg slots (amsg.c) instead of
 * MPI tags.
 *
 * One instance per block root.  Per outer iteration the driver calls
 *   msp_cvd_data_received()  for every newer neighbour iterate   (receive_data_dependency, :600-632)
 *   msp_cvd_step(under)      = comm_async_convDetection_prime (:10-210)
 *                              + receive_partial_CV (:280-330) + receive_verification (:332-365)
 *                              + receive_response (:367-393) + receive_verdict (:395-433)
 * and stops when the state is FINISHED.
 *
 * Faithful to the reference, including two behaviours worth knowing:
 *  - in WAIT4VERIFICATION and VERIFICATION the reference tests the POINTER
 *    `UnderThreashold == PETSC_FALSE` (conv_detection_prime.c:76, :87, :150),
 *    never true, so a block that crossed back above its threshold during the
 *    verification phase does not veto it.  strict = 1 tests the value instead.
 *  - the spanning tree of the reference is the two block roots (build_spanning_tree,
 *    conv_detection.c:180-196); here it is the chain of nb blocks (b-1, b+1), of
 *    which 2 blocks is the reference's case.  Each (source, kind) pair is drained
 *    to its newest message, as the reference's Iprobe/Recv loops do for its one
 *    neighbour.
 */
#include <stdlib.h>
#include <string.h>

#include "msplit.h"
#include "msplit_internal.h"

#define CVD_MAX 8

enum { RESP_NEG = -1, RESP_NEUTRAL = 0, RESP_POS = 1 };
enum { VERDICT_NEG = -1, VERDICT_POS = 1 };

struct msp_cvd {
  msp_amsg *am;
  int32_t rank, strict;
  int32_t nnb, nb[CVD_MAX];     /* spanning-tree neighbours */
  int32_t ndep, dep[CVD_MAX];   /* data dependencies */
  int32_t state, phase_tag;
  int32_t elected, local_cv, partial_cv_sent, response_sent;
  int32_t pp_begin, pp_end, nb_not_recvd;
  int32_t responses[CVD_MAX], received_pcv[CVD_MAX];
  int32_t newer_dep[CVD_MAX], last_iter[CVD_MAX];
  int32_t under;
};

static int cerr(int code, const char *msg) {
  mspi_set_error(code, "%s", msg);
  return code;
}

static void reinitialize_pseudo_period(msp_cvd *c) {
  c->pp_begin = 0;
  c->pp_end = 0;
  for (int d = 0; d < c->ndep; ++d) c->newer_dep[d] = 0;
}

static void initialize_state(msp_cvd *c) {
  c->nb_not_recvd = c->nnb;
  for (int i = 0; i < c->nnb; ++i) c->received_pcv[i] = 0;
  c->elected = 0;
  c->local_cv = 0;
  c->partial_cv_sent = 0;
  reinitialize_pseudo_period(c);
  c->state = MSP_CVD_NORMAL;
}

static void initialize_verification(msp_cvd *c) {
  reinitialize_pseudo_period(c);
  c->phase_tag++;
  for (int i = 0; i < c->nnb; ++i) c->responses[i] = RESP_NEUTRAL;
  c->response_sent = 0;
}

static int all_newer(const msp_cvd *c) {
  for (int d = 0; d < c->ndep; ++d)
    if (!c->newer_dep[d]) return 0;
  return 1;
}

static int count_responses(const msp_cvd *c, int value) {
  int k = 0;
  for (int i = 0; i < c->nnb; ++i) k += c->responses[i] == value;
  return k;
}

static int send2(msp_cvd *c, int dst, int kind, int a, int b, int n) {
  const int32_t v[2] = {a, b};
  return msp_amsg_send(c->am, dst, kind, v, n, NULL, 0);
}

int msp_cvd_create(msp_amsg *am, int32_t rank, int32_t nnb, const int32_t *nb, int32_t ndep, const int32_t *dep,
                   int32_t strict, msp_cvd **out) {
  if (!am || !out || (nnb && !nb) || (ndep && !dep)) return cerr(MSP_ERR_ARG_NULL, "NULL argument");
  if (nnb < 0 || nnb > CVD_MAX || ndep < 0 || ndep > CVD_MAX) return cerr(MSP_ERR_ARG_OUTOFRANGE, "too many neighbours");
  msp_cvd *c = (msp_cvd *)calloc(1, sizeof(msp_cvd));
  if (!c) return cerr(MSP_ERR_MEM, "allocation failed");
  c->am = am;
  c->rank = rank;
  c->strict = strict ? 1 : 0;
  c->nnb = nnb;
  c->ndep = ndep;
  if (nnb) memcpy(c->nb, nb, (size_t)nnb * sizeof(int32_t));
  if (ndep) memcpy(c->dep, dep, (size_t)ndep * sizeof(int32_t));
  for (int d = 0; d < ndep; ++d) c->last_iter[d] = -1; /* VecSet(LastIteration_global, -1) */
  initialize_state(c);
  c->phase_tag = 0;
  *out = c;
  return MSP_SUCCESS;
}

int msp_cvd_destroy(msp_cvd **pc) {
  if (!pc || !*pc) return MSP_SUCCESS;
  free(*pc);
  *pc = NULL;
  return MSP_SUCCESS;
}

int msp_cvd_get_state(const msp_cvd *c, int32_t *state, int32_t *phase_tag) {
  if (!c) return cerr(MSP_ERR_ARG_NULL, "cvd is NULL");
  if (state) *state = c->state;
  if (phase_tag) *phase_tag = c->phase_tag;
  return MSP_SUCCESS;
}

int msp_cvd_get_info(const msp_cvd *c, int32_t *info, int32_t n) {
  if (!c || !info) return cerr(MSP_ERR_ARG_NULL, "NULL argument");
  const int32_t v[8] = {c->state, c->phase_tag, c->elected, c->local_cv,
                        c->pp_begin, c->pp_end, c->nb_not_recvd, c->partial_cv_sent};
  for (int i = 0; i < n && i < 8; ++i) info[i] = v[i];
  return MSP_SUCCESS;
}

/* receive_data_dependency (conv_detection_prime.c:600-632): take an iterate of
 * dependency d when it is newer than the last one taken and, during a
 * verification phase, when it carries the current phase tag. */
int msp_cvd_data_received(msp_cvd *c, int32_t d, int32_t src_tag, int32_t src_iter, int32_t *accept) {
  if (!c || !accept) return cerr(MSP_ERR_ARG_NULL, "NULL argument");
  if (d < 0 || d >= c->ndep) return cerr(MSP_ERR_ARG_OUTOFRANGE, "dependency index");
  *accept = 0;
  if (c->last_iter[d] < src_iter && (c->state != MSP_CVD_VERIFICATION || src_tag == c->phase_tag)) {
    c->last_iter[d] = src_iter;
    c->newer_dep[d] = 1;
    *accept = 1;
  }
  return MSP_SUCCESS;
}

static int send_verification_all(msp_cvd *c, int except) {
  for (int i = 0; i < c->nnb; ++i) {
    if (c->nb[i] == except) continue;
    int rc = send2(c, c->nb[i], MSP_AMSG_VERIFICATION, c->phase_tag, 0, 1);
    if (rc) return rc;
  }
  return MSP_SUCCESS;
}

static int send_verdict_all(msp_cvd *c, int verdict, int except) {
  for (int i = 0; i < c->nnb; ++i) {
    if (c->nb[i] == except) continue;
    int rc = send2(c, c->nb[i], MSP_AMSG_VERDICT, c->phase_tag, verdict, 2);
    if (rc) return rc;
  }
  return MSP_SUCCESS;
}

/* comm_async_convDetection_prime (conv_detection_prime.c:10-210) */
static int conv_detection(msp_cvd *c) {
  int rc = MSP_SUCCESS;
  const int under_in_verif = c->strict ? c->under : 1; /* see the header: the reference never sees "false" */
  if (c->state == MSP_CVD_NORMAL) {
    if (!c->under) {
      reinitialize_pseudo_period(c);
    } else if (!c->pp_begin) {
      c->pp_begin = 1;
    } else if (c->pp_end) {
      c->local_cv = 1;
      if (c->nb_not_recvd == 0) {
        c->elected = 1;
        initialize_verification(c);
        if ((rc = send_verification_all(c, -1))) return rc;
        c->state = MSP_CVD_VERIFICATION;
      } else if (c->nb_not_recvd == 1) {
        for (int i = 0; i < c->nnb; ++i) {
          if (!c->received_pcv[i]) {
            if ((rc = send2(c, c->nb[i], MSP_AMSG_PARTIAL_CV, c->phase_tag, 0, 1))) return rc;
            break;
          }
        }
        c->partial_cv_sent = 1;
        c->state = MSP_CVD_WAIT4VERIFICATION;
      }
    } else if (all_newer(c)) {
      c->pp_end = 1;
    }
  } else if (c->state == MSP_CVD_WAIT4VERIFICATION) {
    if (!under_in_verif) c->local_cv = 0;
  } else if (c->state == MSP_CVD_VERIFICATION) {
    if (c->elected) {
      if (!under_in_verif || !c->local_cv || count_responses(c, RESP_NEG) > 0) {
        c->phase_tag++;
        if ((rc = send_verdict_all(c, VERDICT_NEG, -1))) return rc;
        initialize_state(c);
      } else if (c->pp_end) {
        if (count_responses(c, RESP_NEUTRAL) == 0) {
          if (count_responses(c, RESP_NEG) == 0) {
            if ((rc = send_verdict_all(c, VERDICT_POS, -1))) return rc;
            c->state = MSP_CVD_FINISHED;
          } else {
            c->phase_tag++;
            if ((rc = send_verdict_all(c, VERDICT_NEG, -1))) return rc;
            initialize_state(c);
          }
        }
      } else if (all_newer(c)) {
        c->pp_end = 1;
      }
    } else if (!c->response_sent) {
      if (!under_in_verif || !c->local_cv || count_responses(c, RESP_NEG) > 0) {
        for (int i = 0; i < c->nnb; ++i) {
          if (!c->received_pcv[i]) {
            if ((rc = send2(c, c->nb[i], MSP_AMSG_RESPONSE, c->phase_tag, RESP_NEG, 2))) return rc;
            break;
          }
        }
        c->response_sent = 1;
      } else if (c->pp_end) {
        if (count_responses(c, RESP_NEUTRAL) == 1) {
          int asking = -1;
          for (int i = 0; i < c->nnb; ++i) {
            if (c->responses[i] == RESP_NEUTRAL) {
              asking = c->nb[i];
              break;
            }
          }
          const int resp = count_responses(c, RESP_POS) == c->nnb - 1 ? RESP_POS : RESP_NEG;
          if ((rc = send2(c, asking, MSP_AMSG_RESPONSE, c->phase_tag, resp, 2))) return rc;
          c->response_sent = 1;
        }
      } else if (all_newer(c)) {
        c->pp_end = 1;
      }
    }
  }
  return rc;
}

/* receive_partial_CV (:280-330) */
static int receive_partial_cv(msp_cvd *c) {
  for (int i = 0; i < c->nnb; ++i) {
    int32_t v[1], got = 0;
    int rc = msp_amsg_recv(c->am, c->nb[i], MSP_AMSG_PARTIAL_CV, v, 1, NULL, 0, NULL, &got);
    if (rc) return rc;
    if (!got || v[0] != c->phase_tag) continue;
    c->received_pcv[i] = 1;
    c->nb_not_recvd--;
    const int leader = c->rank > c->nb[i] ? c->rank : c->nb[i]; /* choose_leader: PetscMax */
    if (c->nb_not_recvd == 0 && c->partial_cv_sent && leader == c->rank) {
      c->elected = 1;
      initialize_verification(c);
      if ((rc = send_verification_all(c, -1))) return rc;
      c->state = MSP_CVD_VERIFICATION;
    }
  }
  return MSP_SUCCESS;
}

/* receive_verification (:332-365) */
static int receive_verification(msp_cvd *c) {
  for (int i = 0; i < c->nnb; ++i) {
    int32_t v[1], got = 0;
    int rc = msp_amsg_recv(c->am, c->nb[i], MSP_AMSG_VERIFICATION, v, 1, NULL, 0, NULL, &got);
    if (rc) return rc;
    if (!got || v[0] != c->phase_tag + 1) continue;
    initialize_verification(c);
    c->state = MSP_CVD_VERIFICATION;
    if ((rc = send_verification_all(c, c->nb[i]))) return rc;
  }
  return MSP_SUCCESS;
}

/* receive_response (:367-393) */
static int receive_response(msp_cvd *c) {
  for (int i = 0; i < c->nnb; ++i) {
    int32_t v[2], got = 0;
    int rc = msp_amsg_recv(c->am, c->nb[i], MSP_AMSG_RESPONSE, v, 2, NULL, 0, NULL, &got);
    if (rc) return rc;
    if (got && v[0] == c->phase_tag) c->responses[i] = v[1];
  }
  return MSP_SUCCESS;
}

/* receive_verdict (:395-433) */
static int receive_verdict(msp_cvd *c) {
  for (int i = 0; i < c->nnb; ++i) {
    int32_t v[2], got = 0;
    int rc = msp_amsg_recv(c->am, c->nb[i], MSP_AMSG_VERDICT, v, 2, NULL, 0, NULL, &got);
    if (rc) return rc;
    if (!got) continue;
    if (v[1] == VERDICT_POS) {
      c->state = MSP_CVD_FINISHED;
    } else {
      initialize_state(c);
      c->phase_tag = v[0];
    }
    const int32_t fwd[2] = {c->phase_tag, v[1]};
    for (int k = 0; k < c->nnb; ++k) {
      if (c->nb[k] == c->nb[i]) continue;
      if ((rc = msp_amsg_send(c->am, c->nb[k], MSP_AMSG_VERDICT, fwd, 2, NULL, 0))) return rc;
    }
  }
  return MSP_SUCCESS;
}

int msp_cvd_step(msp_cvd *c, int32_t under_threshold) {
  if (!c) return cerr(MSP_ERR_ARG_NULL, "cvd is NULL");
  c->under = under_threshold ? 1 : 0;
  int rc;
  if ((rc = conv_detection(c)) || (rc = receive_partial_cv(c)) || (rc = receive_verification(c)) ||
      (rc = receive_response(c)) || (rc = receive_verdict(c)))
    return rc;
  return MSP_SUCCESS;
}

/* Error codes shared by every native library (libpcmx_cpu comm layer, libpcmx_hip kernels and RCCL transport).
 * Every public entry point returns 0, one of these, or (HIP calls only) a positive hipError_t;
 * pcmx_error_string (libpcmx_hip) names them. Internal transport codes never leave a public function. */
#ifndef PCMX_ERRORS_H
#define PCMX_ERRORS_H

enum {
    PCMX_ERR_ARG = -1,           /* shape / alignment / argument precondition */
    PCMX_ERR_NOT_CONVERGED = -2, /* an iterate-to-fixpoint loop ran out of max_launches with work left */
    PCMX_ERR_TIMEOUT = -3,       /* a bounded wait gave up: device look-back, or the comm watchdog (result invalid) */
    PCMX_ERR_COMM = -4,          /* a transport / collective / bootstrap failed */
    PCMX_ERR_ALLOC = -5          /* host or device allocation failed */
};

/* Public-boundary normalisation of an internal comm return code: 0 and the codes above pass through, anything
 * else (socket errno paths, RCCL result codes, HIP errors inside the transport) becomes PCMX_ERR_COMM. */
static inline int pcmx_comm_rc(int rc) {
    return (rc == 0 || rc == PCMX_ERR_ARG || rc == PCMX_ERR_TIMEOUT || rc == PCMX_ERR_COMM || rc == PCMX_ERR_ALLOC)
               ? rc
               : PCMX_ERR_COMM;
}

#endif

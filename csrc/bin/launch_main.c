/*
 * pcmx_launch — the native `mpirun -n P prog args...` of the framework (ref 2-mpi-region-growing/Makefile:3-4
 * runs `mpirun -n 1 region pic1.bmp`; 1-introduction/mpi.c is started the same way).
 *
 *   pcmx_launch [-n P] [--port PORT] [--addr ADDR] prog [args...]
 *
 * Starts P copies of prog on this node with torchrun's launch contract in the environment
 * (RANK, WORLD_SIZE, LOCAL_RANK, LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT), so one rank drives one MI355X
 * (LOCAL_RANK -> device) and the comm layer bootstraps over TCP on MASTER_ADDR:MASTER_PORT. Every rank runs in
 * its own process group member of the launcher's group; when one rank fails the others are terminated (they
 * would otherwise wait forever on the dead peer) and the launcher exits with the first failing status.
 * The launcher itself never touches the GPU, so fork/exec here is safe.
 */
#include <errno.h>
#include <netinet/in.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

static int free_port(void) {
    int s = socket(AF_INET, SOCK_STREAM, 0);
    if (s < 0) return 29500;
    struct sockaddr_in a;
    memset(&a, 0, sizeof a);
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = 0;
    socklen_t len = sizeof a;
    int port = 29500;
    if (bind(s, (struct sockaddr*)&a, sizeof a) == 0 && getsockname(s, (struct sockaddr*)&a, &len) == 0)
        port = ntohs(a.sin_port);
    close(s);
    return port;
}

static void usage(void) {
    fprintf(stderr, "usage: pcmx_launch [-n P] [--port PORT] [--addr ADDR] prog [args...]\n");
}

static int exit_code(int status) {
    if (WIFEXITED(status)) return WEXITSTATUS(status);
    if (WIFSIGNALED(status)) return 128 + WTERMSIG(status);
    return 1;
}

int main(int argc, char** argv) {
    int n = 1, port = 0, i = 1;
    const char* addr = "127.0.0.1";
    for (; i < argc; ++i) {
        if (!strcmp(argv[i], "-n") || !strcmp(argv[i], "-np")) {
            if (++i >= argc) return usage(), 2;
            n = atoi(argv[i]);
        } else if (!strcmp(argv[i], "--port")) {
            if (++i >= argc) return usage(), 2;
            port = atoi(argv[i]);
        } else if (!strcmp(argv[i], "--addr")) {
            if (++i >= argc) return usage(), 2;
            addr = argv[i];
        } else if (!strcmp(argv[i], "-h") || !strcmp(argv[i], "--help")) {
            return usage(), 0;
        } else {
            break;
        }
    }
    if (i >= argc || n < 1 || n > 1024) return usage(), 2;
    if (!port) port = free_port();
    char** prog = argv + i;

    pid_t* pids = calloc((size_t)n, sizeof(pid_t));
    if (!pids) return 2;
    char buf[32];
    for (int r = 0; r < n; ++r) {
        pid_t p = fork();
        if (p < 0) {
            perror("fork");
            for (int q = 0; q < r; ++q) kill(pids[q], SIGTERM);
            return 2;
        }
        if (p == 0) {
            snprintf(buf, sizeof buf, "%d", r);
            setenv("RANK", buf, 1);
            setenv("LOCAL_RANK", buf, 1);
            snprintf(buf, sizeof buf, "%d", n);
            setenv("WORLD_SIZE", buf, 1);
            setenv("LOCAL_WORLD_SIZE", buf, 1);
            snprintf(buf, sizeof buf, "%d", port);
            setenv("MASTER_PORT", buf, 1);
            setenv("MASTER_ADDR", addr, 1);
            unsetenv("TORCHELASTIC_RUN_ID"); /* the bootstrap port is MASTER_PORT itself here */
            unsetenv("PCMX_PORT");
            execvp(prog[0], prog);
            fprintf(stderr, "pcmx_launch: cannot run %s: %s\n", prog[0], strerror(errno));
            _exit(127);
        }
        pids[r] = p;
    }

    int first_bad = 0, alive = n;
    while (alive > 0) {
        int status = 0;
        pid_t p = waitpid(-1, &status, 0);
        if (p < 0) {
            if (errno == EINTR) continue;
            break;
        }
        int r = -1;
        for (int q = 0; q < n; ++q)
            if (pids[q] == p) r = q;
        if (r < 0) continue;
        pids[r] = 0;
        --alive;
        const int code = exit_code(status);
        if (code && !first_bad) {
            first_bad = code;
            fprintf(stderr, "pcmx_launch: rank %d exited with status %d; terminating the other ranks\n", r, code);
            /* give peers a moment to finish on their own (a clean error path), then stop them */
            struct timespec ts = {0, 200 * 1000 * 1000};
            nanosleep(&ts, NULL);
            for (int q = 0; q < n; ++q)
                if (pids[q] > 0) kill(pids[q], SIGTERM);
        }
    }
    free(pids);
    return first_bad;
}

/*
 * 8-bit grayscale BMP reader/writer (component C1).
 * Behaviour parity: ref 2-mpi-region-growing/bmp.c:6-47 (writer) and :49-71 (reader), headers bmp.h:6-30.
 *  - writer emits a 14-B file header + 40-B BITMAPINFOHEADER + 256-entry gray palette + pixels + 2 pad
 *    bytes; pixel offset 1078; file_size field = w*h + 56 exactly as the reference computes it.
 *  - deviation (B13): every header byte is defined (creator fields zeroed, trailing pad zeroed), so the
 *    output is byte-for-byte reproducible run to run.
 *  - reader takes width@18, height@22, pixel offset@10 and reads w*h bytes, ignoring row padding.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "pcmx_cpu.h"

static void put_u16(unsigned char* p, unsigned v) { p[0] = (unsigned char)v; p[1] = (unsigned char)(v >> 8); }
static void put_u32(unsigned char* p, unsigned v) {
    for (int i = 0; i < 4; ++i) p[i] = (unsigned char)(v >> (8 * i));
}
static unsigned get_u32(const unsigned char* p) {
    return (unsigned)p[0] | ((unsigned)p[1] << 8) | ((unsigned)p[2] << 16) | ((unsigned)p[3] << 24);
}

int pcmx_write_bmp_path(const char* path, const unsigned char* data, int width, int height) {
    enum { HDR = 54, PAL = 1024 };
    unsigned char head[HDR + PAL];
    memset(head, 0, sizeof head);
    head[0] = 'B';
    head[1] = 'M';
    put_u32(head + 2, (unsigned)(width * height + 54 + 2)); /* reference file_size formula */
    put_u32(head + 10, HDR + PAL);                          /* pixel offset 1078 */
    put_u32(head + 14, 40);
    put_u32(head + 18, (unsigned)width);
    put_u32(head + 22, (unsigned)height);
    put_u16(head + 26, 1);
    put_u16(head + 28, 8);
    put_u32(head + 34, (unsigned)(width * height));
    put_u32(head + 46, 256);
    for (int c = 0; c < 256; ++c) {
        unsigned char* e = head + HDR + 4 * c;
        e[0] = e[1] = e[2] = (unsigned char)c;
    }
    FILE* fp = fopen(path, "wb");
    if (!fp) return -1;
    const unsigned char pad[2] = {0, 0};
    size_t n = (size_t)width * (size_t)height;
    int ok = fwrite(head, 1, sizeof head, fp) == sizeof head && fwrite(data, 1, n, fp) == n &&
             fwrite(pad, 1, 2, fp) == 2;
    ok = (fclose(fp) == 0) && ok;
    return ok ? 0 : -2;
}

void write_bmp(unsigned char* data, int width, int height) {
    if (pcmx_write_bmp_path("out.bmp", data, width, height) != 0) fprintf(stderr, "write_bmp: cannot write out.bmp\n");
}

unsigned char* pcmx_read_bmp_dims(const char* path, int* width, int* height) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return NULL;
    unsigned char hdr[26];
    if (fread(hdr, 1, sizeof hdr, fp) != sizeof hdr || hdr[0] != 'B' || hdr[1] != 'M') {
        fclose(fp);
        return NULL;
    }
    int w = (int)get_u32(hdr + 18), h = (int)get_u32(hdr + 22);
    unsigned off = get_u32(hdr + 10);
    if (h < 0) h = -h;
    if (w <= 0 || h <= 0 || (long long)w * h > (1LL << 31)) {
        fclose(fp);
        return NULL;
    }
    size_t n = (size_t)w * (size_t)h;
    unsigned char* px = (unsigned char*)malloc(n);
    if (!px || fseek(fp, (long)off, SEEK_SET) != 0 || fread(px, 1, n, fp) != n) {
        free(px);
        fclose(fp);
        return NULL;
    }
    fclose(fp);
    if (width) *width = w;
    if (height) *height = h;
    return px;
}

unsigned char* read_bmp(char* filename) { return pcmx_read_bmp_dims(filename, NULL, NULL); }

void pcmx_free(void* p) { free(p); }

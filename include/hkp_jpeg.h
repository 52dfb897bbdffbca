/* hkp_jpeg.h — hybrid JPEG decode for the device data path.
 *
 * Replaces the per-sample `cv2.imread(path)` of the reference's dataset
 * (/root/reference/src/dataset.py:71, KeypointsDataset.__getitem__): the
 * sequential half of a baseline JPEG decode (marker parsing, Huffman entropy
 * decoding of the quantised DCT coefficients) runs on the host in
 * libhkpjpeg.so (plain C, no GPU runtime: it is safe in forked loader workers);
 * the data-parallel half (dequantisation, the 8x8 inverse DCT, chroma
 * upsampling, YCbCr -> BGR) runs on the GPU in libhulkkp.so
 * (hkp_jpeg_reconstruct).  Output: uint8 [n][H][W][3] BGR, bit-identical to
 * libjpeg-turbo's default decode (islow IDCT, fancy upsampling), i.e. to what
 * cv2.imread returns for the same file.
 *
 * Supported: 8-bit baseline / extended-sequential Huffman JPEGs (SOF0, SOF1)
 * with one interleaved scan (or one grayscale component), 1 or 3 components,
 * chroma subsampling 4:4:4, 4:2:2 (h2v1), 4:2:0 (h2v2), restart intervals.
 * Progressive, arithmetic-coded, 12-bit, CMYK / Adobe-RGB and multi-scan
 * sequential files are rejected with HKPJ_ERR_UNSUPPORTED (the caller decodes
 * those on the host).
 */
#ifndef HKP_JPEG_H
#define HKP_JPEG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HKPJ_OK 0
#define HKPJ_ERR_FORMAT (-1)       /* not a JPEG / truncated headers */
#define HKPJ_ERR_UNSUPPORTED (-2)  /* a JPEG this decoder does not take */
#define HKPJ_ERR_CORRUPT (-3)      /* entropy-coded data inconsistent */
#define HKPJ_ERR_ARG (-4)

/* Geometry of one image's coefficient set.  Component c holds bw[c] x bh[c]
 * coefficient blocks (the MCU-padded grid of an interleaved scan; ceil(W/8) x
 * ceil(H/8) for a single-component scan) of which the first dw[c] x dh[c]
 * samples are image data (dw = ceil(W * hs / hmax), dh = ceil(H * vs / vmax)).
 * Blocks are stored component after component, row-major, 64 int16 in natural
 * (row-major 8x8) order; block (bx, by) of component c is at
 * blk_off[c] + by * bw[c] + bx. */
typedef struct hkpj_geom {
    int32_t width, height, ncomp;
    int32_t hs[3], vs[3];        /* sampling factors */
    int32_t hmax, vmax;
    int32_t bw[3], bh[3];        /* coefficient blocks per row / column */
    int32_t dw[3], dh[3];        /* real (downsampled) sample width / height */
    int32_t tq[3];               /* quantisation table index of each component */
    int32_t restart_interval;    /* MCUs per restart interval, 0: none */
    int64_t blk_off[3];          /* first block of each component */
    int64_t nblocks;             /* all components */
} hkpj_geom;

/* Parse the headers of data[0:size) up to the first scan: fills *g.  Returns
 * HKPJ_OK or a negative HKPJ_ERR_*; hkpj_last_error() says why (per thread). */
int hkpj_probe(const uint8_t* data, int64_t size, hkpj_geom* g);

/* Entropy-decode the whole image: coefs = int16 [g->nblocks][64] (natural
 * order, not yet dequantised), qt = uint16 [g->ncomp][64] (each component's
 * quantisation table, natural order).  g must come from hkpj_probe of the same
 * bytes. */
int hkpj_decode(const uint8_t* data, int64_t size, const hkpj_geom* g, int16_t* coefs, uint16_t* qt);

const char* hkpj_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* HKP_JPEG_H */

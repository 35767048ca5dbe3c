/*
 * lpcnet_synth.c -- file-driven C caller of the drop-in boundary: the
 * `-synthesis` mode of the reference's demo (src/lpcnet_demo.c:202-219,
 * USE_WEIGHTS_FILE build) written against include/lpcnet.h only.
 *
 *   lpcnet_synth <weights.bin> <features.f32> <output.pcm>
 *
 * weights.bin   weight blob (src/write_lpcnet_weights.c format, int8 or fp32)
 * features.f32  NB_TOTAL_FEATURES (36) native floats per 10 ms frame, as
 *               `lpcnet_demo -features` writes them; the first NB_FEATURES
 *               (20) are used (lpcnet_demo.c:213-215)
 * output.pcm    16 kHz mono native int16, LPCNET_FRAME_SIZE samples per frame
 *
 * Exit status: 0 ok, 1 runtime failure (message on stderr), 2 usage.
 * Links against liblpcnet_mi355x.so; nothing here knows about HIP.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lpcnet.h"

static unsigned char *read_file(const char *path, int *len)
{
  FILE *f = fopen(path, "rb");
  unsigned char *buf;
  long n;
  if (!f) return NULL;
  if (fseek(f, 0, SEEK_END) != 0 || (n = ftell(f)) < 0 || fseek(f, 0, SEEK_SET) != 0 || n > 0x7fffffffL) {
    fclose(f);
    return NULL;
  }
  buf = (unsigned char *)malloc(n > 0 ? (size_t)n : 1);
  if (buf && fread(buf, 1, (size_t)n, f) != (size_t)n) {
    free(buf);
    buf = NULL;
  }
  fclose(f);
  *len = (int)n;
  return buf;
}

int main(int argc, char **argv)
{
  unsigned char *blob;
  int len = 0, frames = 0, rc = 0;
  FILE *fin, *fout;
  LPCNetState *net;

  if (argc != 4) {
    fprintf(stderr, "usage: %s <weights.bin> <features.f32> <output.pcm>\n", argv[0]);
    return 2;
  }
  blob = read_file(argv[1], &len);
  if (!blob) {
    fprintf(stderr, "cannot read weights %s\n", argv[1]);
    return 1;
  }
  fin = fopen(argv[2], "rb");
  if (!fin) {
    fprintf(stderr, "cannot open features %s\n", argv[2]);
    free(blob);
    return 1;
  }
  fout = fopen(argv[3], "wb");
  if (!fout) {
    fprintf(stderr, "cannot open output %s\n", argv[3]);
    fclose(fin);
    free(blob);
    return 1;
  }

  net = lpcnet_create();
  if (!net || lpcnet_load_model(net, blob, len) != 0) {
    fprintf(stderr, "lpcnet_load_model failed (%s)\n", argv[1]);
    rc = 1;
  }
  /* the blob was copied to the device: the caller may release it now */
  free(blob);
  while (rc == 0) {
    float in_features[NB_TOTAL_FEATURES];
    float features[NB_FEATURES];
    short pcm[LPCNET_FRAME_SIZE];
    size_t got = fread(in_features, sizeof(in_features[0]), NB_TOTAL_FEATURES, fin);
    if (feof(fin) || got != NB_TOTAL_FEATURES) break;
    memcpy(features, in_features, sizeof(features));
    lpcnet_synthesize(net, features, pcm, LPCNET_FRAME_SIZE);
    if (fwrite(pcm, sizeof(pcm[0]), LPCNET_FRAME_SIZE, fout) != LPCNET_FRAME_SIZE) {
      fprintf(stderr, "write failed\n");
      rc = 1;
    }
    frames++;
  }
  if (rc == 0) fprintf(stderr, "%d frames synthesised\n", frames);
  if (net) lpcnet_destroy(net);
  fclose(fin);
  if (fclose(fout) != 0) rc = 1;
  return rc;
}

// Native.java -- JNI entry points of the MI355X LZMA path (jni/lzma_jni.c over
// include/lzma_mi355x.h), used by the drop-in Encoder and Decoder of this package.
// Java 1.6 source level, as the reference builds (pom.xml:67-68).
package SevenZip.Compression.LZMA;

import java.io.IOException;
import java.io.InputStream;

final class Native {
    static final int LZMA_OK = 0;
    static final int LZMA_E_DATA = -5;

    static {
        System.loadLibrary("lzma_mi355x_jni");
        if (!init(Integer.getInteger("lzma.mi355x.devices", 1).intValue())) {
            // the GPU path has no CPU fallback (DESIGN.md section 1)
            throw new UnsatisfiedLinkError("no MI355X device for lzma.mi355x.devices");
        }
    }

    private Native() {
    }

    static native boolean init(int deviceMask);

    /** Encoder.Code on in[0..len): the raw range-coder stream, no header. */
    static native byte[] encode(byte[] in, int len, int dict, int fb, int mf, int lc, int lp, int pb, boolean eos);

    /** Decoder.Code on in[0..len); status[0] = LZMA_OK or LZMA_E_DATA (Code returns false), in
     *  which case the bytes are those the reference had flushed (whole OutWindow windows). */
    static native byte[] decode(byte[] props, byte[] in, int len, long outSize, int[] status);

    /** Encoder.Code on each chunk in[offs[i]..offs[i+1]) over the device mask; returns the packed
     *  layout of the encoded streams in out (N + 1 offsets). */
    static native long[] encodeBatch(byte[] in, long[] offs, byte[] out,
                                     int dict, int fb, int mf, int lc, int lp, int pb, boolean eos);

    /** The sliced encode of in[0..len) (lzma_enc_session_*): a handle for the calls below. */
    static native long sessionBegin(byte[] in, int len, int dict, int fb, int mf, int lc, int lp, int pb, boolean eos);

    /** At least bytes more input parsed and coded; pos[0] = input consumed, pos[1] = output bytes
     *  final so far; true once the stream is flushed. */
    static native boolean sessionStep(long h, long bytes, long[] pos);

    /** Final output bytes [from, from + len) into dst[0..len). */
    static native void sessionOutput(long h, long from, byte[] dst, int len);

    static native void sessionEnd(long h);

    /** The whole of in: Encoder.Code reads its input to EOF (InWindow.java:47-56). */
    static byte[] readAll(InputStream in, int[] len) throws IOException {
        byte[] buf = new byte[1 << 16];
        int n = 0;
        for (;;) {
            if (n == buf.length) {
                if (buf.length == Integer.MAX_VALUE) {
                    throw new IOException("stream longer than a Java array (2 GiB); encode it as independent chunks");
                }
                byte[] bigger = new byte[(int) Math.min(Integer.MAX_VALUE, 2L * buf.length)];
                System.arraycopy(buf, 0, bigger, 0, n);
                buf = bigger;
            }
            int r = in.read(buf, n, buf.length - n);
            if (r < 0) {
                break;
            }
            n += r;
        }
        len[0] = n;
        return buf;
    }
}

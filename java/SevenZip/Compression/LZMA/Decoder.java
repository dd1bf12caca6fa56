// Decoder.java -- drop-in for SevenZip.Compression.LZMA.Decoder (Decoder.java:12-319
// of rfalke/lzma-java): same public surface; Code runs on the MI355X through the JNI
// shim (Native). Java 1.6 source level (pom.xml:67-68).
//
// Departure: Code consumes inStream to EOF before decoding, where the reference's
// RangeDecoder reads lazily (RangeDecoder.java:19-25) and leaves bytes after the
// stream unread. Callers that place data after an LZMA stream must frame it
// (LzmaAlone and LzmaBench do not: one stream per file / buffer).
package SevenZip.Compression.LZMA;

import java.io.IOException;
import java.io.InputStream;
import java.io.OutputStream;

public class Decoder {
    private byte[] _props;

    public Decoder() {
    }

    /** Decoder.SetDecoderProperties (Decoder.java:303-318). */
    public boolean SetDecoderProperties(byte... properties) {
        if (properties.length < 5) {
            return false;
        }
        final int val = properties[0] & 0xFF;
        final int lc = val % 9;
        final int remainder = val / 9;
        final int lp = remainder % 5;
        final int pb = remainder / 5;
        int dictionarySize = 0;
        for (int i = 0; i < 4; i++) {
            dictionarySize += ((int) (properties[1 + i]) & 0xFF) << (i * 8);
        }
        if (lc > Base.kNumLitContextBitsMax || lp > 4 || pb > Base.kNumPosStatesBitsMax) {   // SetLcLpPb :172-182
            return false;
        }
        if (dictionarySize < 0) {   // SetDictionarySize :160-170
            return false;
        }
        _props = new byte[5];
        System.arraycopy(properties, 0, _props, 0, 5);
        return true;
    }

    /** Decoder.Code (Decoder.java:205-301): false on corrupt data, with the bytes the
     *  reference had flushed by then (whole OutWindow windows, OutWindow.java:63-73)
     *  written to outStream; outSize < 0 decodes until the end marker. */
    public boolean Code(InputStream inStream, OutputStream outStream, long outSize) throws IOException {
        if (_props == null) {
            throw new IllegalStateException("SetDecoderProperties first");
        }
        int[] n = new int[1];
        byte[] src = Native.readAll(inStream, n);
        int[] status = new int[1];
        byte[] dst = Native.decode(_props, src, n[0], outSize, status);
        outStream.write(dst);
        outStream.flush();
        return status[0] == Native.LZMA_OK;
    }
}

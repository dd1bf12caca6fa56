// Encoder.java -- drop-in for SevenZip.Compression.LZMA.Encoder (Encoder.java:16-1185
// of rfalke/lzma-java): same public surface and setter semantics; Code runs on the
// MI355X through the JNI shim (Native). Java 1.6 source level (pom.xml:67-68).
package SevenZip.Compression.LZMA;

import SevenZip.ICodeProgress;

import java.io.IOException;
import java.io.InputStream;
import java.io.OutputStream;

public class Encoder {
    private static final int EMatchFinderTypeBT2 = 0;
    private static final int EMatchFinderTypeBT4 = 1;
    private static final int kDefaultDictionaryLogSize = 22;
    private static final int kNumFastBytesDefault = 0x20;

    // Encoder field defaults (Encoder.java:135-172)
    private int _dictionarySize = 1 << kDefaultDictionaryLogSize;
    private int _numFastBytes = kNumFastBytesDefault;
    private int _matchFinderType = EMatchFinderTypeBT4;
    private int _numLiteralContextBits = 3;
    private int _numLiteralPosStateBits = 0;
    private int _posStateBits = 2;
    private boolean _writeEndMark = false;

    public Encoder() {
    }

    /** A no-op in the reference (Encoder.java:1127-1133). */
    public static boolean SetAlgorithm(int algorithm) {
        return true;
    }

    public boolean SetDictionarySize(int dictionarySize) {   // Encoder.java:1135-1146
        final int kDicLogSizeMaxCompress = 29;
        if (dictionarySize < (1 << Base.kDicLogSizeMin) || dictionarySize > (1 << kDicLogSizeMaxCompress)) {
            return false;
        }
        _dictionarySize = dictionarySize;
        return true;
    }

    public boolean SetNumFastBytes(int numFastBytes) {   // Encoder.java:1148-1154
        if (numFastBytes < 5 || numFastBytes > Base.kMatchMaxLen) {
            return false;
        }
        _numFastBytes = numFastBytes;
        return true;
    }

    public boolean SetMatchFinder(int matchFinderIndex) {   // Encoder.java:1156-1167
        if (matchFinderIndex < 0 || matchFinderIndex > 2) {
            return false;
        }
        _matchFinderType = matchFinderIndex;   // 2 (bt4b) codes as bt4 on the device, as in the reference
        return true;
    }

    public boolean SetLcLpPb(int lc, int lp, int pb) {   // Encoder.java:1169-1180
        if (lp < 0 || lp > Base.kNumLitPosStatesBitsEncodingMax || lc < 0 || lc > Base.kNumLitContextBitsMax
                || pb < 0 || pb > Base.kNumPosStatesBitsEncodingMax) {
            return false;
        }
        _numLiteralPosStateBits = lp;
        _numLiteralContextBits = lc;
        _posStateBits = pb;
        return true;
    }

    public void SetEndMarkerMode(boolean endMarkerMode) {   // Encoder.java:1182-1184
        _writeEndMark = endMarkerMode;
    }

    public void WriteCoderProperties(OutputStream outStream) throws IOException {   // Encoder.java:1079-1085
        outStream.write((_posStateBits * 5 + _numLiteralPosStateBits) * 9 + _numLiteralContextBits);
        for (int i = 0; i < 4; i++) {
            outStream.write(_dictionarySize >> (8 * i));
        }
    }

    /** Input bytes per device launch of a long stream's sliced encode (lzma_enc_session_*). */
    static final int kSliceBytes = 16 << 20;

    /** Encoder.Code (Encoder.java:1064-1077): reads inStream to EOF, writes the raw stream;
     *  inSize/outSize are ignored as in the reference (Encoder.java:1046). A stream longer than
     *  one slice is encoded slice by slice (the same bytes): each slice's final output goes to
     *  outStream as it is produced and progress is reported after every slice, as the reference
     *  writes while it codes and reports per block (Encoder.java:1069-1073); a shorter one in one
     *  call, with progress reported once at the end (no output bit depends on it). */
    public void Code(InputStream inStream, OutputStream outStream, long inSize, long outSize,
                     ICodeProgress progress) throws IOException {
        int[] n = new int[1];
        byte[] src = Native.readAll(inStream, n);
        if (n[0] > kSliceBytes) {
            long h = Native.sessionBegin(src, n[0], _dictionarySize, _numFastBytes, _matchFinderType,
                    _numLiteralContextBits, _numLiteralPosStateBits, _posStateBits, _writeEndMark);
            try {
                long[] pos = new long[2];
                long written = 0;
                byte[] buf = new byte[1 << 20];
                boolean done;
                do {
                    done = Native.sessionStep(h, kSliceBytes, pos);
                    while (written < pos[1]) {
                        int k = (int) Math.min(buf.length, pos[1] - written);
                        Native.sessionOutput(h, written, buf, k);
                        outStream.write(buf, 0, k);
                        written += k;
                    }
                    if (progress != null) {
                        progress.SetProgress(pos[0], pos[1]);
                    }
                } while (!done);
            } finally {
                Native.sessionEnd(h);
            }
            outStream.flush();
            return;
        }
        byte[] enc = Native.encode(src, n[0], _dictionarySize, _numFastBytes, _matchFinderType,
                _numLiteralContextBits, _numLiteralPosStateBits, _posStateBits, _writeEndMark);
        outStream.write(enc);
        outStream.flush();   // RangeEncoder.FlushStream (RangeEncoder.java:31-36): flushed, not closed
        if (progress != null) {
            progress.SetProgress(n[0], enc.length);
        }
    }
}

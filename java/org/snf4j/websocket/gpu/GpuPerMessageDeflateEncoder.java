/*
 * The permessage-deflate encoder (PerMessageDeflateEncoder.java:39-100 over
 * DeflateEncoder.java:62-104) on the MI355X.  In the encoder's device batch
 * (wsg_enc_batcher_set_deflate: the k_defl_* kernels ahead of the frame encode) when
 * it directly precedes a GpuFrameEncoder, which is where PerMessageDeflateExtension
 * puts it ("permessage-deflate-encoder" after "ws-encoder",
 * PerMessageDeflateExtension.java:303-313); the deflater state, its window and hash
 * arrays then live in the native batcher, per session, and every compressed payload is
 * byte-identical to java.util.zip.Deflater's.  Otherwise the wrapped reference encoder
 * runs, with its own zlib deflater and session-event handling.
 */
package org.snf4j.websocket.gpu;

import java.util.List;

import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.core.codec.IEncoder;
import org.snf4j.core.codec.IEventDrivenCodec;
import org.snf4j.core.handler.SessionEvent;
import org.snf4j.core.session.ISession;
import org.snf4j.websocket.extensions.compress.PerMessageDeflateEncoder;
import org.snf4j.websocket.frame.Frame;

public class GpuPerMessageDeflateEncoder implements IEncoder<Frame, Frame>, IEventDrivenCodec, GpuStage {

	final int level;
	final boolean noContext;
	private final PerMessageDeflateEncoder fallback;
	private boolean batched;

	public GpuPerMessageDeflateEncoder(int compressionLevel, boolean noContext, PerMessageDeflateEncoder fallback) {
		if (compressionLevel < 0 || compressionLevel > 9)
			throw new IllegalArgumentException("Invalid compressionLevel: " + compressionLevel + " (expected: 0-9)");
		this.level = compressionLevel;
		this.noContext = noContext;
		this.fallback = fallback != null ? fallback : new PerMessageDeflateEncoder(compressionLevel, noContext);
	}

	@Override
	public Class<Frame> getInboundType() {
		return Frame.class;
	}

	@Override
	public Class<Frame> getOutboundType() {
		return Frame.class;
	}

	@Override
	public void setBatched() {
		batched = true;
	}

	@Override
	public boolean isBatched() {
		return batched;
	}

	@Override
	public void encode(ISession session, Frame frame, List<Frame> out) throws Exception {
		if (batched)
			out.add(frame);  // (compressed in the encoder's device batch)
		else
			fallback.encode(session, frame, out);
	}

	@Override
	public void added(ISession session, ICodecPipeline pipeline) {
		fallback.added(session, pipeline);
	}

	@Override
	public void event(ISession session, SessionEvent event) {
		fallback.event(session, event);  // (the batched deflater is dropped by GpuFrameEncoder's slot reset)
	}

	@Override
	public void removed(ISession session, ICodecPipeline pipeline) {
		fallback.removed(session, pipeline);
	}
}

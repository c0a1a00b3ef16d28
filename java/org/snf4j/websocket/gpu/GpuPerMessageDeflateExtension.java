/*
 * permessage-deflate with the MI355X inflate: PerMessageDeflateExtension
 * (PerMessageDeflateExtension.java:45-328) negotiates exactly as the reference
 * (this class delegates offer / acceptOffer / validateResponse / response to it),
 * and the negotiated extension's updateDecoders puts the reference
 * PerMessageDeflateDecoder after "ws-decoder" (:316-326), which is then wrapped
 * in a GpuPerMessageDeflateDecoder under the same key.  The decoder's noContext is
 * the negotiated one: the client's no_context_takeover for a server, the server's
 * for a client (:321-325), read back from the response parameters.  Compression:
 * updateEncoders puts the reference PerMessageDeflateEncoder after "ws-encoder"
 * (:303-313), which is then wrapped in a GpuPerMessageDeflateEncoder under the same key
 * ("permessage-deflate-encoder") with the negotiated noContext (the server's
 * server_no_context_takeover for a server, the client's for a client, :310) and the
 * compression level; behind a GpuFrameEncoder it compresses in that encoder's device
 * batch.  The level: the one given here (PerMessageDeflateExtension keeps its own
 * private), 6 by default as PerMessageDeflateExtension() (:144-146).
 */
package org.snf4j.websocket.gpu;

import java.util.List;

import org.snf4j.core.codec.ICodec;
import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.websocket.extensions.IExtension;
import org.snf4j.websocket.extensions.InvalidExtensionException;
import org.snf4j.websocket.IWebSocketSessionConfig;
import org.snf4j.websocket.extensions.compress.PerMessageDeflateDecoder;
import org.snf4j.websocket.extensions.compress.PerMessageDeflateEncoder;
import org.snf4j.websocket.extensions.compress.PerMessageDeflateExtension;
import org.snf4j.websocket.extensions.compress.PerMessageDeflateExtension.NoContext;

public class GpuPerMessageDeflateExtension implements IExtension {

	private static final String CLIENT_NO_CONTEXT = "client_no_context_takeover";
	private static final String SERVER_NO_CONTEXT = "server_no_context_takeover";

	private static final int DEFAULT_LEVEL = 6;

	private final PerMessageDeflateExtension delegate;
	/** null: not negotiated yet; true: the server side (acceptOffer); false: the client side */
	private final Boolean server;
	private final int compressionLevel;

	/** The delegate built with the given compression level. */
	public GpuPerMessageDeflateExtension(PerMessageDeflateExtension delegate, int compressionLevel) {
		this(delegate, null, compressionLevel);
	}

	/** The delegate built with the default compression level (6). */
	public GpuPerMessageDeflateExtension(PerMessageDeflateExtension delegate) {
		this(delegate, null, DEFAULT_LEVEL);
	}

	/** As PerMessageDeflateExtension(compressionLevel, compressNoContext, decompressNoContext). */
	public GpuPerMessageDeflateExtension(int compressionLevel, NoContext compressNoContext,
			NoContext decompressNoContext) {
		this(new PerMessageDeflateExtension(compressionLevel, compressNoContext, decompressNoContext), null,
				compressionLevel);
	}

	public GpuPerMessageDeflateExtension() {
		this(new PerMessageDeflateExtension(), null, DEFAULT_LEVEL);
	}

	private GpuPerMessageDeflateExtension(PerMessageDeflateExtension delegate, Boolean server, int compressionLevel) {
		this.delegate = delegate;
		this.server = server;
		this.compressionLevel = compressionLevel;
	}

	@Override
	public String getName() {
		return delegate.getName();
	}

	@Override
	public Object getGroupId() {
		return delegate.getGroupId();
	}

	@Override
	public IExtension acceptOffer(List<String> offer) throws InvalidExtensionException {
		IExtension e = delegate.acceptOffer(offer);
		return e == null ? null
				: new GpuPerMessageDeflateExtension((PerMessageDeflateExtension) e, Boolean.TRUE, compressionLevel);
	}

	@Override
	public IExtension validateResponse(List<String> response) throws InvalidExtensionException {
		IExtension e = delegate.validateResponse(response);
		return e == null ? null
				: new GpuPerMessageDeflateExtension((PerMessageDeflateExtension) e, Boolean.FALSE, compressionLevel);
	}

	@Override
	public List<String> offer() {
		return delegate.offer();
	}

	@Override
	public List<String> response() {
		return delegate.response();
	}

	@Override
	public void updateEncoders(ICodecPipeline pipeline) {
		delegate.updateEncoders(pipeline);
		ICodec<?, ?> c = pipeline.get(PerMessageDeflateExtension.PERMESSAGE_DEFLATE_ENCODER);
		if (c instanceof PerMessageDeflateEncoder) {
			List<String> r = delegate.response();
			boolean noContext = r.contains(Boolean.TRUE.equals(server) ? SERVER_NO_CONTEXT : CLIENT_NO_CONTEXT);
			GpuPerMessageDeflateEncoder g = new GpuPerMessageDeflateEncoder(compressionLevel, noContext,
					(PerMessageDeflateEncoder) c);
			pipeline.replace(PerMessageDeflateExtension.PERMESSAGE_DEFLATE_ENCODER,
					PerMessageDeflateExtension.PERMESSAGE_DEFLATE_ENCODER, g);
			ICodec<?, ?> w = pipeline.get(IWebSocketSessionConfig.WEBSOCKET_ENCODER);
			if (w instanceof GpuFrameEncoder)
				((GpuFrameEncoder) w).attachDeflate(g);
		}
	}

	@Override
	public void updateDecoders(ICodecPipeline pipeline) {
		delegate.updateDecoders(pipeline);
		ICodec<?, ?> c = pipeline.get(PerMessageDeflateExtension.PERMESSAGE_DEFLATE_DECODER);
		if (c instanceof PerMessageDeflateDecoder) {
			List<String> r = delegate.response();
			boolean noContext = r.contains(Boolean.TRUE.equals(server) ? CLIENT_NO_CONTEXT : SERVER_NO_CONTEXT);
			pipeline.replace(PerMessageDeflateExtension.PERMESSAGE_DEFLATE_DECODER,
					PerMessageDeflateExtension.PERMESSAGE_DEFLATE_DECODER,
					new GpuPerMessageDeflateDecoder(noContext, (PerMessageDeflateDecoder) c));
		}
	}
}
